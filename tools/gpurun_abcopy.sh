# A/B: counters-only memset / copy-back when spans are off (off2) against the full span region
# (off) and the code before the spans (qc); then one rank's share of the 8-way split over 300 steps.
set -o pipefail
VARIANTS="off2:off2 off:off qc:qc:RT_FRAMES_IN_FLIGHT=4,RT_FINISH_FRAC=20" REPS=3 EXTRA=--no-isolated bash tools/gpurun_ab4.sh || exit 1
VARIANTS="d:off2 t512:off2:RT_TAIL_RAYS=524288 ff15:off2:RT_FINISH_FRAC=15 ff30:off2:RT_FINISH_FRAC=30 q8f6:off2:RT_HW_QUEUES=8,RT_FRAMES_IN_FLIGHT=6" REPS=2 STEPS=300 EXTRA="--no-isolated --emulate-ranks 8" bash tools/gpurun_ab4.sh
