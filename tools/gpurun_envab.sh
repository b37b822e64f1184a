# A/B of environment variants on the default bench workload (alternating runs, one library):
#   VARIANTS="base: g1280:RT_SHADE_BLOCKS=1280" REPS=3 bash tools/gpurun_envab.sh
# each variant is name:VAR=value[,VAR=value...] (empty after the colon = the defaults)
set -o pipefail
mkdir -p gpurun_out
for i in $(seq ${REPS:-3}); do
  for v in ${VARIANTS}; do
    name=${v%%:*}; envs=${v#*:}
    timeout -k 10 200 env ${envs//,/ } python -u bench.py --no-cpu --steps ${STEPS:-48} --warmup 4 $EXTRA > gpurun_out/eab_$name$i.log 2>&1 || { tail -c 1500 gpurun_out/eab_$name$i.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
r=d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], 'frac', r['frac'], [(k['kernel'][:12], k['launch_ms']) for k in r['kernels']], d['config']['stage_ms'])" gpurun_out/eab_$name$i.log "$name $i"
  done
done
