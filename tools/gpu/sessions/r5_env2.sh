# HSA signal waits by polling instead of interrupts (host wake-up latency at the timed region's
# closing synchronize)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
AB_ENVS="noint:HSA_ENABLE_INTERRUPT=0" bash tools/gpu/ab_libs.sh gpurun_out/r5_env2 3
