# Final round-3 profile set with the product library (TAG=r03h) and the C3r line.
set -o pipefail
mkdir -p gpurun_out
TAG=r03h bash tools/gpurun_profile.sh || exit 1
timeout -k 10 300 python -u bench.py --scene c3r > gpurun_out/r03h_c3r_bench.json 2> gpurun_out/r03h_c3r_bench.err
rc=$?; cat gpurun_out/r03h_c3r_bench.json; exit $rc
