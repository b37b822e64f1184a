#!/bin/bash
# round 6: the configs table with the final code (tools/configs.sh: every BASELINE config with its PMC passes)
mkdir -p gpurun_out
timeout -k 10 1150 bash tools/configs.sh > gpurun_out/configs.txt 2>&1 || exit 4
