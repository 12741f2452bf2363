# A/B of the uniform-layout metadata fast path against the previous commit.
set -e
mkdir -p gpurun_out
B=boringssl_amd/csrc/build
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config config2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/f_c2_main_$rep.log 2>&1
  BSSL_AMD_LIB=$PWD/$B/ab_prevgcm/libbssl_amd.so timeout -k 10 200 python bench.py --config config2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/f_c2_prev_$rep.log 2>&1
  timeout -k 10 200 python bench.py --config config3 --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/f_c3_main_$rep.log 2>&1
  BSSL_AMD_LIB=$PWD/$B/ab_prevcha/libbssl_amd.so timeout -k 10 200 python bench.py --config config3 --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/f_c3_prev_$rep.log 2>&1
done
timeout -k 10 200 python bench.py --config config4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/f_c4_main_1.log 2>&1
BSSL_AMD_LIB=$PWD/$B/ab_prevgcm/libbssl_amd.so timeout -k 10 200 python bench.py --config config4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/f_c4_prev_1.log 2>&1
