# per-block start / end of every step kernel (tools/step_timeline.py --by-mod K:<blocks>)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5_blocks; mkdir -p $O
timeout -k 10 150 python tools/step_timeline.py --by-mod tail:609 --by-mod conv12_fwd:256 --by-mod fc1_fwd:256 \
  --by-mod fc1_bwd_head:216 --by-mod conv_bwd4:256 --json $O/timeline.json > $O/timeline.txt 2>&1; rc=$?
head -12 $O/timeline.txt; exit $rc
