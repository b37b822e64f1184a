#!/bin/bash
# Per-rank throughput of an N-way tile split, emulated in one process (no gather):
#   EMUL="2 4 8" FIFS="0 2 4" bash tools/gpurun_emul.sh  -> gpurun_out/emul_<N>_<fif>.json
mkdir -p gpurun_out
for n in ${EMUL:-2 4 8}; do
  for f in ${FIFS:-0}; do
    timeout -k 10 120 python bench.py --no-cpu --steps ${STEPS:-32} --emulate-ranks $n --frames-in-flight $f $EXTRA > gpurun_out/emul_${n}_${f}.json 2> gpurun_out/emul_${n}_${f}.err || { echo "emul $n $f failed"; tail -5 gpurun_out/emul_${n}_${f}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['config']['frames_in_flight'])" gpurun_out/emul_${n}_${f}.json $n $f
  done
done
