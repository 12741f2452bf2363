# Round-5 final evidence on one GPU: every config's bench line with its digest
# check (config 2 with the CPU baseline), the table-free engine's lines of the
# AES-GCM configs, open lines, the 2-rank rehearsal, then the FETCH/WRITE
# calibration copies, rocprofv3 kernel traces (steady-state means) and the
# PMC passes of the bench commands, and the end-to-end PCIe rates.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${RUN:-r5final}
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
step bench 600 python bench.py
for c in configG config3 config3x config4 config5 configS; do
  step bench_$c 300 python bench.py --config $c --no-cpu-baseline
done
for c in config2 configG config4 config5; do
  step bs_$c 300 env BSSL_AMD_GCM_MODE=bs python bench.py --config $c --no-cpu-baseline
done
step bench_config2_open 300 python bench.py --op open --no-cpu-baseline
step bench_config3_open 300 python bench.py --config config3 --op open --no-cpu-baseline
step rehearse2 300 env BSSL_AMD_REHEARSE_DEVICES=1 python bench.py --gpus 2 --no-cpu-baseline
O=$O/prof CONFIGS="config2 configG config3 config4 config5" PASSES="calib stats pmc" bash tools/profile.sh || exit 1
step e2e_config2 300 python3 tools/e2e_bench.py --config config2 --records 262144 --chunk 8192
step e2e_config3 300 python3 tools/e2e_bench.py --config config3 --records 1048576 --chunk 65536
