#!/bin/bash
# Per-rank load balance of an N-way tile split: every rank's share rendered alone (bench.py
# --emulate-ranks N --emulate-rank r); TILES selects tile sizes
mkdir -p gpurun_out
N=${N:-8}
for t in ${TILES:-64 32}; do
  for r in $(seq 0 $((N - 1))); do
    log=gpurun_out/bal_t${t}_r$r.log
    timeout -k 10 200 python -u bench.py --no-cpu --steps 32 --warmup 4 --tile $t --emulate-ranks $N --emulate-rank $r > $log 2>&1 || { tail -c 1500 $log; exit 1; }
    python -c "
import json
d=json.loads([x for x in open('$log') if x.startswith('{')][-1])
print('tile $t rank $r', d['value'], d['ms_per_step'])"
  done
done
