cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5_bm
timeout -k 10 150 python tools/step_timeline.py --by-mod conv_bwd4:4 --by-mod conv12_fwd:4 --by-mod fc1_bwd_head:50 --by-mod tail:1 --json gpurun_out/r5_bm/timeline.json > gpurun_out/r5_bm/timeline.txt 2>&1; rc=$?; cat gpurun_out/r5_bm/timeline.txt; exit $rc
