#!/bin/bash
# round 6 closing measurement with the final defaults: the round's profiles (bench line with PMC and CPU
# baseline, rocprof kernel stats alone / in flight, roofline check), then the configs table
mkdir -p gpurun_out
TAG=r06 timeout -k 10 1000 bash tools/profile_round.sh > gpurun_out/profile_round.log 2>&1 || exit 3
timeout -k 10 1400 bash tools/configs.sh > gpurun_out/configs.txt 2>&1 || exit 4
