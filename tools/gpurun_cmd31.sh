# finish-kernel path chunk (RT_FCHUNK) at N = 1 and the 8-way share, final kernels
VARIANTS="base RT_FCHUNK=16 RT_FCHUNK=64" REPS=2 bash tools/gpurun_multiab.sh || exit 1
VARIANTS="base RT_FCHUNK=16 RT_FCHUNK=64" REPS=2 EXTRA="--emulate-ranks 8 --steps 48" bash tools/gpurun_multiab.sh
