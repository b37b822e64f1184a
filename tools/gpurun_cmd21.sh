# four-slot finish threshold at the 2- and 4-way rank shares: 768K (default) against 512K
VARIANTS="base RT_TAIL_RAYS=524288" REPS=2 EXTRA="--emulate-ranks 2 --steps 48" bash tools/gpurun_multiab.sh || exit 1
VARIANTS="base RT_TAIL_RAYS=524288" REPS=2 EXTRA="--emulate-ranks 4 --steps 48" bash tools/gpurun_multiab.sh
