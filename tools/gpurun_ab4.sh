# A/B of library variants and environment settings, alternating runs on one box (default bench
# workload).  VARIANTS = "name:lib[:ENV=v,ENV2=v]" entries; lib = ab_<lib>.so.  PARITY = a lib whose
# golden / C3g parity tests run first (the product library is restored afterwards).
set -o pipefail
mkdir -p gpurun_out
cp metal4-raytracing_amd/librt_hip.so /tmp/librt_keep.so
restore() { cp /tmp/librt_keep.so metal4-raytracing_amd/librt_hip.so; }
for lib in ${PARITY}; do
  cp ab_$lib.so metal4-raytracing_amd/librt_hip.so
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "golden or glass_dragon or light_types or c3g" > gpurun_out/parity_$lib.log 2>&1 || { tail -30 gpurun_out/parity_$lib.log; restore; exit 1; }
  tail -2 gpurun_out/parity_$lib.log
done
for i in $(seq ${REPS:-3}); do
  for v in ${VARIANTS}; do
    name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; envs=""; [ "$rest" != "$lib" ] && envs=${rest#*:}
    cp ab_$lib.so metal4-raytracing_amd/librt_hip.so
    env ${envs//,/ } timeout -k 10 200 python -u bench.py --no-cpu --steps ${STEPS:-48} --warmup 4 $EXTRA > gpurun_out/lab_$name$i.log 2>&1 || { tail -c 1500 gpurun_out/lab_$name$i.log; restore; exit 1; }
    python3 -c "
import json,sys
d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], 'frac', r['frac'], [(k['kernel'][:12], k['launch_ms'], k.get('launch_ms_device'), k['nodes_per_ray']) for k in r['kernels']], d['config']['stage_ms'])" gpurun_out/lab_$name$i.log "$name $i"
  done
done
restore
