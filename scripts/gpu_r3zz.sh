# Round-3 final check at HEAD: the whole GPU suite, smoke, the default bench line.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r3zz bash scripts/gpu_tests.sh
