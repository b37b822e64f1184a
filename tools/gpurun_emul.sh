#!/bin/bash
# Per-rank throughput of an N-way tile split, emulated in one process (no gather):
#   EMUL="2 4 8" FIFS="0 2 4" HWQS="4 8" bash tools/gpurun_emul.sh  -> gpurun_out/emul_<N>_<fif>_<hwq>.json
# (HWQS: hardware queues per run via RT_HW_QUEUES, which bench.py turns into GPU_MAX_HW_QUEUES; 4 = HIP's default)
mkdir -p gpurun_out
for n in ${EMUL:-2 4 8}; do
  for f in ${FIFS:-0}; do
   for q in ${HWQS:-4}; do
    o=gpurun_out/emul_${n}_${f}_${q}
    RT_HW_QUEUES=$q timeout -k 10 120 python bench.py --no-cpu --steps ${STEPS:-32} --emulate-ranks $n --frames-in-flight $f $EXTRA > $o.json 2> $o.err || { echo "emul $n $f $q failed"; tail -5 $o.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], sys.argv[4], d['value'], d['ms_per_step'], d['config']['frames_in_flight'])" $o.json $n $f $q
   done
  done
done
