// Issue cost of the integer VALU instructions of the ChaCha20 and Poly1305
// inner loops on gfx950: cycles per wave-instruction per SIMD with 1 and 4
// waves per SIMD, 8 independent chains per wave (s_memtime around a fixed
// unrolled stream).  Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kIters = 256;

#define BODY8(INSN)                                                   \
  asm volatile(INSN(0) INSN(1) INSN(2) INSN(3) INSN(4) INSN(5) INSN(6) INSN(7) \
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), \
                 "+v"(r[6]), "+v"(r[7]) : "v"(a), "v"(b) : "s40", "s41");

// 64-bit register pairs for the mad/shift cases.
#define BODY8_64(INSN)                                                  \
  asm volatile(INSN(0) INSN(1) INSN(2) INSN(3) INSN(4) INSN(5) INSN(6) INSN(7) \
               : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), \
                 "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b) : "s40", "s41");

#define I_ADD(i) "v_add_u32 %" #i ", %" #i ", %8\n"
#define I_XOR(i) "v_xor_b32 %" #i ", %" #i ", %8\n"
#define I_ALIGNBIT(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 16\n"
#define I_BITOP3(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %9 bitop3:0x96\n"
#define I_MULLO(i) "v_mul_lo_u32 %" #i ", %" #i ", %8\n"
#define I_MULHI(i) "v_mul_hi_u32 %" #i ", %" #i ", %8\n"
#define I_MAD64(i) "v_mad_u64_u32 %" #i ", s[40:41], %8, %9, %" #i "\n"
#define I_SHR64(i) "v_lshrrev_b64 %" #i ", 26, %" #i "\n"
#define I_ADD64(i) "v_lshl_add_u64 %" #i ", %" #i ", 0, %" #i "\n"
#define I_PERM(i) "v_perm_b32 %" #i ", %" #i ", %" #i ", %9\n"
#define I_ALIGNBYTE(i) "v_alignbyte_b32 %" #i ", %" #i ", %" #i ", 2\n"
#define I_LSHLOR(i) "v_lshl_or_b32 %" #i ", %" #i ", 7, %8\n"
#define I_XAD(i) "v_xad_u32 %" #i ", %" #i ", %8, %9\n"
#define I_ADD3(i) "v_add3_u32 %" #i ", %" #i ", %8, %9\n"
#define I_LSHL(i) "v_lshlrev_b32 %" #i ", 7, %" #i "\n"
#define I_XOR_SDWA(i) "v_xor_b32_sdwa %" #i ", %" #i ", %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n"
#define I_PK_ADD16(i) "v_pk_add_u16 %" #i ", %" #i ", %8 op_sel:[1,1] op_sel_hi:[0,0]\n"

// ChaCha quarter-round-like dependent triples (add, xor, rotate) on ILP
// independent chains.
#define QSTEP(i) "v_add_u32 %" #i ", %" #i ", %8\n v_xor_b32 %" #i ", %" #i ", %9\n v_alignbit_b32 %" #i ", %" #i ", %" #i ", 16\n"
#define QBODY4 asm volatile(QSTEP(0) QSTEP(1) QSTEP(2) QSTEP(3) : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]) : "v"(a), "v"(b));
#define QBODY8 asm volatile(QSTEP(0) QSTEP(1) QSTEP(2) QSTEP(3) QSTEP(4) QSTEP(5) QSTEP(6) QSTEP(7) : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]) : "v"(a), "v"(b));

template <int K>
__global__ void rate(uint64_t *out, uint32_t a, uint32_t b) {
  uint32_t r[8];
  uint64_t w[8];
  for (int i = 0; i < 8; i++) { r[i] = threadIdx.x + i; w[i] = threadIdx.x * 3ull + i; }
  if (K == 16) for (int i = 0; i < 8; i++) r[i] = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; it++) {
    if (K == 0) { BODY8(I_ADD) BODY8(I_ADD) BODY8(I_ADD) BODY8(I_ADD) }
    if (K == 1) { BODY8(I_XOR) BODY8(I_XOR) BODY8(I_XOR) BODY8(I_XOR) }
    if (K == 2) { BODY8(I_ALIGNBIT) BODY8(I_ALIGNBIT) BODY8(I_ALIGNBIT) BODY8(I_ALIGNBIT) }
    if (K == 3) { BODY8(I_BITOP3) BODY8(I_BITOP3) BODY8(I_BITOP3) BODY8(I_BITOP3) }
    if (K == 4) { BODY8(I_MULLO) BODY8(I_MULLO) BODY8(I_MULLO) BODY8(I_MULLO) }
    if (K == 5) { BODY8(I_MULHI) BODY8(I_MULHI) BODY8(I_MULHI) BODY8(I_MULHI) }
    if (K == 6) { BODY8_64(I_MAD64) BODY8_64(I_MAD64) BODY8_64(I_MAD64) BODY8_64(I_MAD64) }
    if (K == 7) { BODY8_64(I_SHR64) BODY8_64(I_SHR64) BODY8_64(I_SHR64) BODY8_64(I_SHR64) }
    if (K == 8) { BODY8_64(I_ADD64) BODY8_64(I_ADD64) BODY8_64(I_ADD64) BODY8_64(I_ADD64) }
    if (K == 9) { BODY8(I_PERM) BODY8(I_PERM) BODY8(I_PERM) BODY8(I_PERM) }
    if (K == 10) { BODY8(I_ALIGNBYTE) BODY8(I_ALIGNBYTE) BODY8(I_ALIGNBYTE) BODY8(I_ALIGNBYTE) }
    if (K == 11) { BODY8(I_LSHLOR) BODY8(I_LSHLOR) BODY8(I_LSHLOR) BODY8(I_LSHLOR) }
    if (K == 12) { BODY8(I_XAD) BODY8(I_XAD) BODY8(I_XAD) BODY8(I_XAD) }
    if (K == 13) { BODY8(I_ADD3) BODY8(I_ADD3) BODY8(I_ADD3) BODY8(I_ADD3) }
    if (K == 14) { BODY8(I_LSHL) BODY8(I_LSHL) BODY8(I_LSHL) BODY8(I_LSHL) }
    // power probes: same instruction, operands that toggle all bits / none
    if (K == 15) { BODY8(I_XOR) BODY8(I_XOR) BODY8(I_XOR) BODY8(I_XOR) }
    if (K == 16) { BODY8(I_ALIGNBIT) BODY8(I_ALIGNBIT) BODY8(I_ALIGNBIT) BODY8(I_ALIGNBIT) }
    // 32 instructions per iteration in both: ILP 4 (the QR interleave of one
    // ChaCha block) vs ILP 8 (two blocks interleaved); order within a step
    // keeps each chain's add -> xor -> rotate dependent.
    if (K == 17) { QBODY4 QBODY4 asm volatile("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n" : "+v"(r[5]) : "v"(a)); }
    if (K == 19) { BODY8(I_XOR_SDWA) BODY8(I_XOR_SDWA) BODY8(I_XOR_SDWA) BODY8(I_XOR_SDWA) }
    if (K == 20) { BODY8(I_PK_ADD16) BODY8(I_PK_ADD16) BODY8(I_PK_ADD16) BODY8(I_PK_ADD16) }
    if (K == 18) { QBODY8 asm volatile("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n" : "+v"(r[5]) : "v"(a)); }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t acc = 0;
  for (int i = 0; i < 8; i++) acc += r[i] + w[i];
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
  if (acc == 0x123456789ull) out[0] = acc;
}

int main() {
  const char *names[] = {"v_add_u32", "v_xor_b32", "v_alignbit_b32", "v_bitop3_b32", "v_mul_lo_u32",
                         "v_mul_hi_u32", "v_mad_u64_u32", "v_lshrrev_b64", "v_lshl_add_u64",
                         "v_perm_b32", "v_alignbyte_b32", "v_lshl_or_b32", "v_xad_u32", "v_add3_u32",
                         "v_lshlrev_b32", "v_xor_b32 ~0", "v_alignbit(0)", "QR ILP4(+8 add)", "QR ILP8(+8 add)",
                         "v_xor_b32_sdwa", "v_pk_add_u16"};
  uint64_t *d;
  CK(hipMalloc(&d, 1 << 20));
  uint64_t h[4096];
  // s_memtime counts shader-clock cycles; the ratio to v_add_u32 under the
  // same occupancy is reported beside them.
  for (int waves = 1; waves <= 4; waves *= 4) {
    double base = 0;
    for (int k = 0; k < 21; k++) {
      for (int rep = 0; rep < 2; rep++) {
        // one workgroup per CU, `waves` waves per SIMD
        const int threads = 256 * waves;
        switch (k) {
          case 0: rate<0><<<256, threads>>>(d, 3, 5); break;
          case 1: rate<1><<<256, threads>>>(d, 3, 5); break;
          case 2: rate<2><<<256, threads>>>(d, 3, 5); break;
          case 3: rate<3><<<256, threads>>>(d, 3, 5); break;
          case 4: rate<4><<<256, threads>>>(d, 3, 5); break;
          case 5: rate<5><<<256, threads>>>(d, 3, 5); break;
          case 6: rate<6><<<256, threads>>>(d, 3, 5); break;
          case 7: rate<7><<<256, threads>>>(d, 3, 5); break;
          case 8: rate<8><<<256, threads>>>(d, 3, 5); break;
          case 9: rate<9><<<256, threads>>>(d, 3, 0x05040706); break;
          case 10: rate<10><<<256, threads>>>(d, 3, 5); break;
          case 11: rate<11><<<256, threads>>>(d, 3, 5); break;
          case 12: rate<12><<<256, threads>>>(d, 3, 5); break;
          case 13: rate<13><<<256, threads>>>(d, 3, 5); break;
          case 14: rate<14><<<256, threads>>>(d, 3, 5); break;
          case 15: rate<15><<<256, threads>>>(d, 0xffffffffu, 5); break;
          case 16: rate<16><<<256, threads>>>(d, 3, 5); break;
          case 17: rate<17><<<256, threads>>>(d, 3, 5); break;
          case 18: rate<18><<<256, threads>>>(d, 3, 5); break;
          case 19: rate<19><<<256, threads>>>(d, 3, 5); break;
          case 20: rate<20><<<256, threads>>>(d, 3, 5); break;
        }
        CK(hipDeviceSynchronize());
      }
      const int nw = 256 * 4 * waves;
      CK(hipMemcpy(h, d, nw * 8, hipMemcpyDeviceToHost));
      double s = 0;
      for (int i = 0; i < nw; i++) s += h[i];
      s /= nw;
      const double instr = 32.0 * kIters;                    // per wave
      const double cyc = s / instr;
      if (k == 0) base = s;
      printf("waves/SIMD %d  %-16s ~%.2f cycles per wave-instruction per wave (x%.2f v_add)  => SIMD %.2f cyc/instr\n",
             waves, names[k], cyc, s / base, cyc / waves);
    }
  }
  return 0;
}
