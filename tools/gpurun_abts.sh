# A/B of the device-clock launch spans: per-block, per-XCD-line end stamps (fix) against one
# atomic per wave on one line (new = the library before) and the code before the spans (qc).
# GPU tests of the stamp-reading paths first.
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_inflight.py -x -q --timeout 200 --timeout-method thread > gpurun_out/abts_tests.log 2>&1 || { tail -20 gpurun_out/abts_tests.log; exit 1; }
tail -2 gpurun_out/abts_tests.log
VARIANTS="fix:fix new:new qc:qc:RT_FRAMES_IN_FLIGHT=4,RT_FINISH_FRAC=20" REPS=3 EXTRA=--no-isolated bash tools/gpurun_ab4.sh
