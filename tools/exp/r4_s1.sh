# Round 4, session 1: per-rank parity of multi-GPU shards on one GPU (the
# bench's own shard layouts vs tests/golden/ref_shard_digests.json), the
# 2-rank rehearsal of the launcher with all-ranks parity, and same-box
# baselines of the round-3 kernels.  Each step has its own limit; a failure
# ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4s1
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/steps.log
  tail -3 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step shards 900 python -u -m pytest tests/test_bench_layout.py -v -m gpu -k shard_of_multi --timeout 300 --timeout-method thread
for c in config2 config4 config5; do
  step rehearse2_$c 600 env BSSL_AMD_REHEARSE_DEVICES=1 python bench.py --gpus 2 --config $c --steps 5 --warmup 2 --no-cpu-baseline
done
for c in config2 configG config4 config5 config3; do
  step base_$c 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline
done
