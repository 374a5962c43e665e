# Several scripts/gpu_ab.sh sets in one GPU call (a box is slow to get; one call amortises it).
# usage: gpurun -- 'SETS="tagA;VARIANTS_A;ARGS_A;STEPS_A;ROUNDS_A@tagB;..." bash scripts/gpu_multi_ab.sh'
#   each set: TAG ; VARIANTS ("|"-separated, as gpu_ab.sh) ; ARGS ; STEPS ; ROUNDS, sets split by "@"
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
IFS='@' read -ra SS <<< "${SETS}"
for set in "${SS[@]}"; do
  IFS=';' read -r tag variants args steps rounds <<< "$set"
  echo "== set $tag"
  TAG="$tag" VARIANTS="$variants" ARGS="$args" STEPS="${steps:-100}" ROUNDS="${rounds:-2}" bash scripts/gpu_ab.sh || exit $?
done
exit 0
