# A round's final evidence on one GPU (RUN names the output dir under
# gpurun_out/): the GPU test suite and smoke, every config's bench line with
# its digest check (config 2 with the CPU baseline), open lines, the table-free
# and mixed engines' lines of the AES-GCM configs, the 2-rank rehearsal, the
# end-to-end PCIe rates, then the FETCH/WRITE calibration copies, rocprofv3
# kernel traces and the PMC passes of the bench commands for both AES-GCM
# engines (tools/profile.sh; summarise with tools/pmc_traffic.py).  Each GPU
# step has its own time limit; the chain stops at the first fault or timeout.
#   RUN=r6final bash tools/exp/final_evidence.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-final}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.log | head -1)" | tee -a $O/steps.log
  [ $rc -eq 0 ] || { tail -3 "$O/$name.log"; exit $rc; }
}
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python bench.py
for c in configG config3 config3x config4 config5 configS; do
  step bench_$c 300 python bench.py --config $c --no-cpu-baseline
done
step bench_config2_open 300 python bench.py --op open --no-cpu-baseline
step bench_config3_open 300 python bench.py --config config3 --op open --no-cpu-baseline
for c in config2 configG config4 config5; do
  step bs_$c 300 env BSSL_AMD_GCM_MODE=bs python bench.py --config $c --no-cpu-baseline
done
step mix6_config2 300 env BSSL_AMD_GCM_MODE=mix6 python bench.py --no-cpu-baseline
step rehearse2 300 env BSSL_AMD_REHEARSE_DEVICES=1 python bench.py --gpus 2 --no-cpu-baseline
step e2e_config2 300 python3 tools/e2e_bench.py --config config2 --records 262144 --chunk 8192
step e2e_config3 300 python3 tools/e2e_bench.py --config config3 --records 1048576 --chunk 65536
O=$O/prof CONFIGS="config2 configG config3 config4 config5" PASSES="calib stats pmc" bash tools/profile.sh || exit 1
O=$O/prof ENGINE=bs CONFIGS="config2 configG config4 config5" PASSES="stats pmc" bash tools/profile.sh || exit 1
