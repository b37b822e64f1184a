#!/bin/bash
# Every config through bench.py + the emulated 2/4/8-way rank shares + one rank of configs[3]
set -o pipefail
bash tools/gpurun_configs.sh || exit 1
EMUL="2 4 8" STEPS=300 EXTRA=--no-isolated bash tools/gpurun_emul.sh || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --width 3840 --height 2160 --spp 16 --steps 6 --warmup 2 --emulate-ranks 8 > gpurun_out/c4r8.log 2>&1 || { tail -c 1500 gpurun_out/c4r8.log; exit 1; }
python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/c4r8.log') if x.startswith('{')][-1]); print('c4 rank8', d['value'], d['ms_per_step'])"
