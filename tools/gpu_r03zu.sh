#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 ./tools/_abl/gdn_prof > gpurun_out/r03zu_gdnprof.txt 2>&1; rc=$?; cat gpurun_out/r03zu_gdnprof.txt; exit $rc
