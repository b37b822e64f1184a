# Isolated-launch roofline + irregular-geometry check: the bench contract test and the C3r parity
# test, the default bench line (with roofline.isolated), and the bench on C3r.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_parity.py -k "bench or real_meshes" -x -v --timeout 300 --timeout-method thread > gpurun_out/iso_tests.log 2>&1
rc=$?; tail -6 gpurun_out/iso_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/iso_bench.json 2> gpurun_out/iso_bench.err
rc=$?; cat gpurun_out/iso_bench.json; tail -3 gpurun_out/iso_bench.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --scene c3r > gpurun_out/iso_c3r.json 2> gpurun_out/iso_c3r.err
rc=$?; cat gpurun_out/iso_c3r.json; tail -3 gpurun_out/iso_c3r.err; exit $rc
