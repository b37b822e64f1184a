# A/B of library variants ab_<name>.so (alternating runs, default bench workload, two frames in flight)
set -o pipefail
mkdir -p gpurun_out
cp metal4-raytracing_amd/librt_hip.so /tmp/librt_keep.so
for i in $(seq ${REPS:-3}); do
  for v in ${LIBS}; do
    cp ab_$v.so metal4-raytracing_amd/librt_hip.so
    timeout -k 10 200 python -u bench.py --no-cpu --steps ${STEPS:-48} --warmup 4 $EXTRA > gpurun_out/lab_$v$i.log 2>&1 || { tail -c 1500 gpurun_out/lab_$v$i.log; cp /tmp/librt_keep.so metal4-raytracing_amd/librt_hip.so; exit 1; }
    python3 -c "
import json,sys
d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], 'frac', r['frac'], [(k['kernel'][:12], k['launch_ms'], k['nodes_per_ray'], k['lds_nodes_per_ray']) for k in r['kernels']], d['config']['stage_ms'])" gpurun_out/lab_$v$i.log "$v $i"
  done
done
cp /tmp/librt_keep.so metal4-raytracing_amd/librt_hip.so
