#!/bin/bash
# AEGIS lab: hand-scheduled asm update step vs production steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02l
mkdir -p $OUT
timeout -k 10 240 ./tools/aegis_lab 16384 > $OUT/aegis_lab.json 2>&1 || { echo LAB_FAILED; tail -20 $OUT/aegis_lab.json; exit 1; }
grep -v '"col' $OUT/aegis_lab.json
