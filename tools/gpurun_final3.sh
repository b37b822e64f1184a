# Round-3 final: the spans-off A/B (off = product library, qc = before the spans), the round's
# profile set (TAG=r03g), the C3r bench line, then the four-slot knob sweep.
set -o pipefail
mkdir -p gpurun_out
VARIANTS="off:off qc:qc:RT_FRAMES_IN_FLIGHT=4,RT_FINISH_FRAC=20" REPS=3 EXTRA=--no-isolated bash tools/gpurun_ab4.sh || exit 1
TAG=r03g bash tools/gpurun_profile.sh || exit 1
timeout -k 10 300 python -u bench.py --scene c3r > gpurun_out/r03g_c3r_bench.json 2> gpurun_out/r03g_c3r_bench.err
rc=$?; cat gpurun_out/r03g_c3r_bench.json; [ $rc -ne 0 ] && exit $rc
bash tools/gpurun_sweep4.sh
