# rank-share tail knobs (8-way emulation) and frames in flight at N = 1
VARIANTS="base RT_TAIL_RAYS=262144 RT_TAIL_RAYS=786432 RT_FINISH_FRAC=15 RT_FINISH_FRAC=25" REPS=2 EXTRA="--emulate-ranks 8 --steps 48" bash tools/gpurun_multiab.sh || exit 1
VARIANTS="base RT_FRAMES_IN_FLIGHT=3" REPS=2 bash tools/gpurun_multiab.sh
