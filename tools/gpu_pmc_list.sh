#!/bin/bash
cd /tmp && export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/pmc_avail.txt 2>&1
echo rc=$?
grep -c . $GRAFT_REPO_ROOT/gpurun_out/pmc_avail.txt
