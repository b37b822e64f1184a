# The scheduling knobs at four frames in flight (C3g default bench, then one rank's share of the
# 8-way split): shade grid, refill threshold, finish chunk, finish shading threshold.
VARIANTS="d:off sh2560:off:RT_SHADE_BLOCKS=2560 sh4096:off:RT_SHADE_BLOCKS=4096 rm4:off:RT_REFILL_MIN=4 rm16:off:RT_REFILL_MIN=16 fc16:off:RT_FCHUNK=16 fc64:off:RT_FCHUNK=64 sm16:off:RT_SHADE_MIN=16 sm32:off:RT_SHADE_MIN=32" REPS=2 EXTRA=--no-isolated bash tools/gpurun_ab4.sh || exit 1
bash tools/gpurun_rank8.sh
