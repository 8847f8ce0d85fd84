#!/bin/bash
# Copy what tools/profile_r03.sh left under gpurun_out/ into profiles/ (run
# here, after the gpurun call): traffic.json + kernel stats of configs 2, 3
# and 5 (tools/traffic.py), bench lines of every config, the GPU suite's
# summary, config 1/4 kernel stats and the k-way probe.
set -e -o pipefail
cd "$(dirname "$0")/.."
for c in 2 3 5; do
  rm -rf profiles/r03_c$c
  python tools/traffic.py gpurun_out/prof_r03_c$c profiles/r03_c$c
  grep '^{' gpurun_out/prof_r03_c$c/bench.json | tail -1 > profiles/r03_final/bench_c$c.json
done
for c in 1 4; do
  grep '^{' gpurun_out/r03/bench_c$c.log | tail -1 > profiles/r03_final/bench_c$c.json
  cp gpurun_out/r03/trace_c$c/run_kernel_stats.csv profiles/r03_final/kernel_stats_c$c.csv
done
tail -3 gpurun_out/r03/gpu_tests.log > profiles/r03_final/gpu_tests.log
cp gpurun_out/r03/scan_probe.json profiles/r03_final/scan_probe.json
cat gpurun_out/r03/lib.md5
