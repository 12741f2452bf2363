set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/al
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu -k "chacha or uniform or baseline or bench_layout or synth or tls or iov or ragged or kat or Sealv" --timeout 300 --timeout-method thread > gpurun_out/t_main.log 2>&1 || { tail -30 gpurun_out/t_main.log; exit 1; }
tail -1 gpurun_out/t_main.log
BSSL_AMD_LIB=$PWD/boringssl_amd/csrc/build/ab_line2/libbssl_amd.so timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "chacha and (uniform or baseline or bench_layout or synth)" --timeout 300 --timeout-method thread > gpurun_out/t_line2.log 2>&1 || { tail -30 gpurun_out/t_line2.log; exit 1; }
tail -1 gpurun_out/t_line2.log
for rep in 1 2; do
 for c in config3 config3x; do
  for al in 128 16; do
   for v in main ab_line2 ab_nocoal2; do
    if [ $v = main ]; then unset BSSL_AMD_LIB; else export BSSL_AMD_LIB=$PWD/boringssl_amd/csrc/build/$v/libbssl_amd.so; fi
    BSSL_AMD_ALIGN=$al timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/al/${c}_${v}_a${al}_$rep.log 2>&1 || exit 1
    echo "$c $v align=$al rep=$rep $(grep -o '"value": [0-9.]*' gpurun_out/al/${c}_${v}_a${al}_$rep.log | head -1)"
   done
  done
 done
done
unset BSSL_AMD_LIB
