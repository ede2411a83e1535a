# conv_bwd4 db_conv2 per chunk row: A/B against HEAD's library (run with HEAD's row geometry)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
AB_ENVS="head:PTO_HIP_LIB=pytorch_operator_amd/_lib/exp_old/head.so,PTO_B2_ROWS=old" TL_ARGS="--by-mod tail:609" \
  bash tools/gpu/ab_libs.sh gpurun_out/r5_b2c 2
