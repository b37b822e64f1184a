set -o pipefail
# Per-rank throughput of an N-way tile split (bench.py --emulate-ranks) across frames-in-flight
# counts.  RANKS / FIFS select the sweep; EXTRA passes more bench flags.
mkdir -p gpurun_out
for r in ${RANKS:-8 4}; do
  for f in ${FIFS:-3 4 5}; do
    log=gpurun_out/${TAG}ranks${r}_fif$f.log
    timeout -k 10 240 python -u bench.py --no-cpu --steps ${STEPS:-32} --warmup 4 --emulate-ranks $r --frames-in-flight $f $EXTRA > $log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -c 1500 $log; exit $rc; }
    python -c "
import json
d=json.loads([x for x in open('$log') if x.startswith('{')][-1])
print('$TAG ranks $r fif $f', d['value'], d['ms_per_step'], d['config']['stage_ms'])"
  done
done
