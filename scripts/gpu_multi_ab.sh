# Several scripts/gpu_ab.sh sets in one GPU call (a box is slow to get; one call amortises it).
# usage: gpurun -- 'SETS_FILE=scripts/ab/<name>.sets bash scripts/gpu_multi_ab.sh'
#   one set per line: TAG ; VARIANTS ("|"-separated, as gpu_ab.sh) ; ARGS ; STEPS ; ROUNDS
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mapfile -t SS < "${SETS_FILE}"
for set in "${SS[@]}"; do
  [ -z "$set" ] && continue
  IFS=';' read -r tag variants args steps rounds <<< "$set"
  echo "== set $tag"
  TAG="$tag" VARIANTS="$variants" ARGS="$args" STEPS="${steps:-100}" ROUNDS="${rounds:-2}" bash scripts/gpu_ab.sh || exit $?
done
exit 0
