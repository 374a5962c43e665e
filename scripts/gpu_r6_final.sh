# Round-6 closing evidence at the final code: rocprofv3 kernel stats + timelines and PMC HBM traffic
# (FETCH_SIZE / WRITE_SIZE, one pass each, summarised by scripts/pmc_summary.py into profiles/pmc_*.json,
# which bench.py reads for roofline.traffic) of the headline (C2/C4), C3, the heavy-tail point and C5.
# usage: gpurun -- 'TAG=r6z SK=k_stream4 bash scripts/gpu_r6_final.sh'   env: PARTS (default all), SK (stream kernel)
set -u
TAG=${TAG:-r6z}
SK=${SK:-k_stream4}
PARTS=${PARTS:-"c2 c3 heavy expand"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
Q="--cpu-seconds 0 --parity 0 --latency-batches 0 --host-calls 0 --expand-steps 0 --c3-steps 0 --sharded-steps 0 --heavy-steps 0"
pmc() {  # name, kernel regex, bench args
  local n=$1 rx=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-include-regex "$rx" --pmc FETCH_SIZE -d gpurun_out/pmc_${TAG}_${n}_fetch -o run --output-format csv -- python3 bench.py "$@" > gpurun_out/pmc_${TAG}_${n}_fetch.log 2>&1 || { echo "pmc fetch $n failed"; return 1; }
  timeout -s KILL 240 rocprofv3 --kernel-include-regex "$rx" --pmc WRITE_SIZE -d gpurun_out/pmc_${TAG}_${n}_write -o run --output-format csv -- python3 bench.py "$@" > gpurun_out/pmc_${TAG}_${n}_write.log 2>&1 || { echo "pmc write $n failed"; return 1; }
  echo "pmc $n ok"
}
for P in $PARTS; do
  case $P in
  c2)
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c2 -o run --output-format csv -- python3 bench.py --steps 40 --warmup 6 $Q > gpurun_out/prof_${TAG}_c2.log 2>&1 || { echo "c2 trace failed"; exit 1; }
    python3 scripts/timeline.py gpurun_out/prof_${TAG}_c2/run_kernel_trace.csv > gpurun_out/timeline_${TAG}_c2.txt || true
    pmc c2 "${SK}|k_resolve|k_back" --steps 6 --warmup 4 $Q || exit 1
    for K in $SK k_resolve k_back; do
      python3 scripts/pmc_summary.py --kernel $K --fetch gpurun_out/pmc_${TAG}_c2_fetch --write gpurun_out/pmc_${TAG}_c2_write --tuples 1e9 --batch 1000000 --preset 0 --inflight 4 --out gpurun_out/pmc_${K}_p0.json > /dev/null || true
    done
    echo "c2 done"
    ;;
  c3)
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c3 -o run --output-format csv -- python3 bench.py --preset 1 --tuples 1e7 --inflight 6 --steps 30 --warmup 6 $Q > gpurun_out/prof_${TAG}_c3.log 2>&1 || { echo "c3 trace failed"; exit 1; }
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c3one -o run --output-format csv -- python3 bench.py --preset 1 --tuples 1e7 --inflight 1 --steps 10 --warmup 3 $Q > gpurun_out/prof_${TAG}_c3one.log 2>&1 || { echo "c3 one-batch trace failed"; exit 1; }
    ANCHOR=k_fsplit python3 scripts/timeline.py gpurun_out/prof_${TAG}_c3one/run_kernel_trace.csv > gpurun_out/timeline_${TAG}_c3.txt || true
    pmc c3 "k_grid_level|${SK}|k_fsplit|k_back|k_resolve" --preset 1 --tuples 1e7 --inflight 6 --steps 6 --warmup 6 $Q || exit 1
    for K in k_grid_level $SK k_fsplit k_back k_resolve; do
      python3 scripts/pmc_summary.py --kernel $K --fetch gpurun_out/pmc_${TAG}_c3_fetch --write gpurun_out/pmc_${TAG}_c3_write --tuples 1e7 --batch 1000000 --preset 1 --inflight 6 --out gpurun_out/pmc_${K}_p1.json > /dev/null || true
    done
    echo "c3 done"
    ;;
  heavy)
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_heavy -o run --output-format csv -- python3 bench.py --heavy-tail --steps 20 --warmup 4 $Q > gpurun_out/prof_${TAG}_heavy.log 2>&1 || { echo "heavy trace failed"; exit 1; }
    python3 scripts/timeline.py gpurun_out/prof_${TAG}_heavy/run_kernel_trace.csv > gpurun_out/timeline_${TAG}_heavy.txt || true
    pmc heavy "k_ms_level|${SK}" --heavy-tail --steps 4 --warmup 4 $Q || exit 1
    for K in k_ms_level $SK; do
      python3 scripts/pmc_summary.py --kernel $K --fetch gpurun_out/pmc_${TAG}_heavy_fetch --write gpurun_out/pmc_${TAG}_heavy_write --tuples 1.2e8 --batch 62500 --preset 0 --inflight 4 --out gpurun_out/pmc_${K}_p0h.json > /dev/null || true
    done
    echo "heavy done"
    ;;
  expand)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_expand -o run --output-format csv -- python3 bench.py --mode expand --inflight 20 --steps 40 --warmup 20 --cpu-seconds 0 --parity-roots 0 --hw-queues 32 > gpurun_out/prof_${TAG}_expand.log 2>&1 || { echo "expand trace failed"; exit 1; }
    python3 scripts/busy.py gpurun_out/prof_${TAG}_expand/run_kernel_trace.csv "k_expand" > gpurun_out/busy_${TAG}_expand.txt || true
    pmc expand "k_expand" --mode expand --inflight 20 --steps 20 --warmup 20 --cpu-seconds 0 --parity-roots 0 --hw-queues 32 || exit 1
    python3 scripts/pmc_summary.py --kernel k_expand --anchor k_expand_lds --fetch gpurun_out/pmc_${TAG}_expand_fetch --write gpurun_out/pmc_${TAG}_expand_write --tuples 1e9 --batch 100000 --preset 0 --inflight 20 --out gpurun_out/pmc_k_expand_p0x.json > /dev/null || true
    echo "expand done"
    ;;
  esac
done
exit 0
