# A/B of the queue-carried path state (bf74367) against the code before it (7e6c31f) and the current
# library, all at four frames in flight with the finish on 20 % of the grid (the default since
# 2a1d281); ab_old.so / ab_qc.so are built from those commits' sources in a git worktree.
VARIANTS="new:new old:old:RT_FRAMES_IN_FLIGHT=4,RT_FINISH_FRAC=20 qc:qc:RT_FRAMES_IN_FLIGHT=4,RT_FINISH_FRAC=20" REPS=3 EXTRA=--no-isolated bash tools/gpurun_ab4.sh
