# One rank's share of the 8-way C3g split (--emulate-ranks 8), the scheduling knobs with the
# round-3 kernels: hardware queues / slots, finish threshold and finish share.
VARIANTS="d:off q8:off:RT_HW_QUEUES=8 q8f6:off:RT_HW_QUEUES=8,RT_FRAMES_IN_FLIGHT=6 t512:off:RT_TAIL_RAYS=524288 t1m:off:RT_TAIL_RAYS=1048576 ff30:off:RT_FINISH_FRAC=30 ff15:off:RT_FINISH_FRAC=15" REPS=2 EXTRA="--no-isolated --emulate-ranks 8" bash tools/gpurun_ab4.sh
