# Frames in flight x hardware queues on the default bench workload (A/B, alternating runs).
set -o pipefail
mkdir -p gpurun_out
VARIANTS="${VARIANTS:-f4:ts:RT_FRAMES_IN_FLIGHT=4 f5:ts:RT_FRAMES_IN_FLIGHT=5 f6:ts:RT_FRAMES_IN_FLIGHT=6 f6q8:ts:RT_FRAMES_IN_FLIGHT=6,RT_HW_QUEUES=8 f8q8:ts:RT_FRAMES_IN_FLIGHT=8,RT_HW_QUEUES=8}" REPS=${REPS:-2} bash tools/gpurun_ab4.sh
