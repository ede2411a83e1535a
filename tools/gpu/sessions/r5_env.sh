# HIP runtime knobs on the stream-launched MNIST step: device-memory kernel arguments on / off,
# one hardware queue
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
AB_ENVS="devk1:HIP_FORCE_DEV_KERNARG=1 devk0:HIP_FORCE_DEV_KERNARG=0 hwq1:GPU_MAX_HW_QUEUES=1" \
  bash tools/gpu/ab_libs.sh gpurun_out/r5_env 2
