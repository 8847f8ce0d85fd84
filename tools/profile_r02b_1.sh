#!/bin/bash
# Round-2b profiles, part 1: config 2 (bench line, trace, PMC passes) + traces of configs 1 and 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CONFIG=2 EXTRA_CONFIGS="1 4" bash tools/profile.sh r02b_c2 || exit 1
echo PART1_OK
