#!/bin/bash
# Producer timing split (spec_probe) for configs 2 and 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02r
mkdir -p $OUT
TBC_PROBE_PRODUCERS_ONLY=1 timeout -k 10 200 python -u tools/spec_probe.py --config 2 --jobs 8 > $OUT/p2.json 2>&1 || { echo P2_FAILED; tail -20 $OUT/p2.json; exit 1; }
cat $OUT/p2.json
TBC_PROBE_PRODUCERS_ONLY=1 timeout -k 10 200 python -u tools/spec_probe.py --config 4 --jobs 10 > $OUT/p4.json 2>&1 || { echo P4_FAILED; tail -20 $OUT/p4.json; exit 1; }
cat $OUT/p4.json
