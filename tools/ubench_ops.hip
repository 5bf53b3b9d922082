// Issue-cost microbenchmark for the non-product VALU ops of the field
// multiply (tools/ubench_int.hip measured the products; its carry rows ran one
// serial VCC chain, so they priced latency, not issue). Every lane runs CH
// independent chains, each with its own carry SGPR pair, so the numbers are
// SIMD issue cycles per wave64 instruction at 8 waves/SIMD; round 4 adds the
// same table at ONE wave per SIMD (the block kernel's regime: a lone wave pays
// an op's issue cost and its dependent latency, nothing hides either) and
// dependent-chain rows for the carry, DPP and 24-bit multiply forms.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_ops.hip -o tools/ubench_ops
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 1024;
constexpr int CH = 8;

struct Stamp { unsigned long long t0, t1, r0, r1; };

// instructions per chain step for each op
static const int NINSTR[] = {1, 1, 1, 1, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 3, 1, 1,
                             1, 1, 1, 1, 2, 1, 1, 1};
static const char* NAMES[] = {
    "v_add_u32",                        // 0
    "v_add_co_u32_e64 (sdst)",          // 1
    "v_addc_co_u32_e64 (own s pair)",   // 2
    "v_mad_u64_u32 (own s pair)",       // 3
    "mad(co)+addc_e64 (own s pair)",    // 4
    "mad(co->vcc)+addc_e32 (vcc)",      // 5
    "v_add3_u32",                       // 6
    "v_lshl_add_u32",                   // 7
    "v_alignbit_b32",                   // 8
    "v_lshrrev_b64",                    // 9
    "v_mov_b32",                        // 10
    "v_and_b32",                        // 11
    "v_cndmask_b32_e64 (fixed mask)",   // 12
    "v_lshl_add_u64",                   // 13
    "v_mad_u64_u32 (no carry use, sdst null)",  // 14
    "add_co+addc_e64 64-bit add (own pairs)",   // 15
    "v_bfe_u32",                        // 16
    "v_mul_u32_u24",                    // 17
    "v_mad_u64_u32 dependent chain (1/lane)",  // 18
    "v_add_u32 dependent chain (1/lane)",      // 19
    "v_add_co_u32_e32 (vcc out)",       // 20
    "v_addc_co_u32_e32 (vcc chain)",    // 21
    "v_cndmask_b32_e32 (vcc)",          // 22
    "v_lshlrev_b32_e32",                // 23
    "v_or_b32_e32",                     // 24
    "v_sub_u32_e32",                    // 25
    "v_add_u32_e64 (VOP3 form)",        // 26
    "v_subb_co_u32_e32 (vcc chain)",    // 27
    "v_xor_b32_e32",                    // 28
    "v_lshrrev_b32_e32",                // 29
    "v_mul_lo_u32",                     // 30
    "mad(co->vcc)+addc_e32, 1 instr apart, no nop",  // 31
    "v_cndmask_b32_e32 (vcc from v_cmp_e32 each 8)",  // 32
    "v_cndmask_b32_e64 (s pair from v_cmp_e64 each 8)",  // 33
    "v_mov_b32_dpp quad_perm (independent)",  // 34
    "v_mad_u32_u24",                    // 35
    "v_mul_hi_u32",                     // 36
    "v_add3_u32 dependent chain (1/lane)",  // 37
    "v_addc_co_u32_e64 dependent SGPR-carry chain + s_nop 1 (1/lane)",  // 38
    "v_mov_b32_dpp dependent chain (1/lane)",  // 39
    "v_mad_u32_u24 dependent chain (1/lane)",  // 40
    "v_lshl_add_u64 dependent chain (1/lane)",  // 41
};

template <int OP>
__global__ void __launch_bounds__(256) kern(uint32_t seed, uint32_t* out, Stamp* st) {
  uint32_t a[CH], h[CH];
  uint64_t acc[CH];
  const uint32_t b = seed ^ threadIdx.x;
#pragma unroll
  for (int k = 0; k < CH; ++k) { a[k] = seed * (k + 3) + threadIdx.x; h[k] = a[k] ^ 0x5555u; acc[k] = a[k]; }
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      if constexpr (OP == 0) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 1) {
        switch (k) {
          case 0: asm volatile("v_add_co_u32_e64 %0, s[20:21], %0, %1" : "+v"(a[k]) : "v"(b) : "s20", "s21"); break;
          case 1: asm volatile("v_add_co_u32_e64 %0, s[22:23], %0, %1" : "+v"(a[k]) : "v"(b) : "s22", "s23"); break;
          case 2: asm volatile("v_add_co_u32_e64 %0, s[24:25], %0, %1" : "+v"(a[k]) : "v"(b) : "s24", "s25"); break;
          case 3: asm volatile("v_add_co_u32_e64 %0, s[26:27], %0, %1" : "+v"(a[k]) : "v"(b) : "s26", "s27"); break;
          case 4: asm volatile("v_add_co_u32_e64 %0, s[28:29], %0, %1" : "+v"(a[k]) : "v"(b) : "s28", "s29"); break;
          case 5: asm volatile("v_add_co_u32_e64 %0, s[30:31], %0, %1" : "+v"(a[k]) : "v"(b) : "s30", "s31"); break;
          case 6: asm volatile("v_add_co_u32_e64 %0, s[56:57], %0, %1" : "+v"(a[k]) : "v"(b) : "s56", "s57"); break;
          case 7: asm volatile("v_add_co_u32_e64 %0, s[34:35], %0, %1" : "+v"(a[k]) : "v"(b) : "s34", "s35"); break;
        }
      } else if constexpr (OP == 2) {
        switch (k) {
          case 0: asm volatile("v_addc_co_u32_e64 %0, s[20:21], %0, %1, s[20:21]" : "+v"(a[k]) : "v"(b) : "s20", "s21"); break;
          case 1: asm volatile("v_addc_co_u32_e64 %0, s[22:23], %0, %1, s[22:23]" : "+v"(a[k]) : "v"(b) : "s22", "s23"); break;
          case 2: asm volatile("v_addc_co_u32_e64 %0, s[24:25], %0, %1, s[24:25]" : "+v"(a[k]) : "v"(b) : "s24", "s25"); break;
          case 3: asm volatile("v_addc_co_u32_e64 %0, s[26:27], %0, %1, s[26:27]" : "+v"(a[k]) : "v"(b) : "s26", "s27"); break;
          case 4: asm volatile("v_addc_co_u32_e64 %0, s[28:29], %0, %1, s[28:29]" : "+v"(a[k]) : "v"(b) : "s28", "s29"); break;
          case 5: asm volatile("v_addc_co_u32_e64 %0, s[30:31], %0, %1, s[30:31]" : "+v"(a[k]) : "v"(b) : "s30", "s31"); break;
          case 6: asm volatile("v_addc_co_u32_e64 %0, s[56:57], %0, %1, s[56:57]" : "+v"(a[k]) : "v"(b) : "s56", "s57"); break;
          case 7: asm volatile("v_addc_co_u32_e64 %0, s[34:35], %0, %1, s[34:35]" : "+v"(a[k]) : "v"(b) : "s34", "s35"); break;
        }
      } else if constexpr (OP == 3) {
        switch (k) {
          case 0: asm volatile("v_mad_u64_u32 %0, s[20:21], %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "s20", "s21"); break;
          case 1: asm volatile("v_mad_u64_u32 %0, s[22:23], %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "s22", "s23"); break;
          case 2: asm volatile("v_mad_u64_u32 %0, s[24:25], %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "s24", "s25"); break;
          case 3: asm volatile("v_mad_u64_u32 %0, s[26:27], %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "s26", "s27"); break;
          case 4: asm volatile("v_mad_u64_u32 %0, s[28:29], %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "s28", "s29"); break;
          case 5: asm volatile("v_mad_u64_u32 %0, s[30:31], %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "s30", "s31"); break;
          case 6: asm volatile("v_mad_u64_u32 %0, s[56:57], %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "s56", "s57"); break;
          case 7: asm volatile("v_mad_u64_u32 %0, s[34:35], %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "s34", "s35"); break;
        }
      } else if constexpr (OP == 4) {
        switch (k) {
          case 0: asm volatile("v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[20:21], %1, 0, s[20:21]" : "+v"(acc[k]), "+v"(h[k]) : "v"(a[k]), "v"(b) : "s20", "s21"); break;
          case 1: asm volatile("v_mad_u64_u32 %0, s[22:23], %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[22:23], %1, 0, s[22:23]" : "+v"(acc[k]), "+v"(h[k]) : "v"(a[k]), "v"(b) : "s22", "s23"); break;
          case 2: asm volatile("v_mad_u64_u32 %0, s[24:25], %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[24:25], %1, 0, s[24:25]" : "+v"(acc[k]), "+v"(h[k]) : "v"(a[k]), "v"(b) : "s24", "s25"); break;
          case 3: asm volatile("v_mad_u64_u32 %0, s[26:27], %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[26:27], %1, 0, s[26:27]" : "+v"(acc[k]), "+v"(h[k]) : "v"(a[k]), "v"(b) : "s26", "s27"); break;
          case 4: asm volatile("v_mad_u64_u32 %0, s[28:29], %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[28:29], %1, 0, s[28:29]" : "+v"(acc[k]), "+v"(h[k]) : "v"(a[k]), "v"(b) : "s28", "s29"); break;
          case 5: asm volatile("v_mad_u64_u32 %0, s[30:31], %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[30:31], %1, 0, s[30:31]" : "+v"(acc[k]), "+v"(h[k]) : "v"(a[k]), "v"(b) : "s30", "s31"); break;
          case 6: asm volatile("v_mad_u64_u32 %0, s[56:57], %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[56:57], %1, 0, s[56:57]" : "+v"(acc[k]), "+v"(h[k]) : "v"(a[k]), "v"(b) : "s56", "s57"); break;
          case 7: asm volatile("v_mad_u64_u32 %0, s[34:35], %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[34:35], %1, 0, s[34:35]" : "+v"(acc[k]), "+v"(h[k]) : "v"(a[k]), "v"(b) : "s34", "s35"); break;
        }
      } else if constexpr (OP == 5) {
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                     : "+v"(acc[k]), "+v"(h[k]) : "v"(a[k]), "v"(b) : "vcc");
      } else if constexpr (OP == 6) {
        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(h[k]));
      } else if constexpr (OP == 7) {
        asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 8) {
        asm volatile("v_alignbit_b32 %0, %1, %0, 29" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 9) {
        asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(acc[k]));
      } else if constexpr (OP == 10) {
        asm volatile("v_mov_b32 %0, %1" : "=v"(a[k]) : "v"(h[(k + 1) % CH]));
        asm volatile("" : "+v"(h[(k + 1) % CH]));
      } else if constexpr (OP == 11) {
        asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 12) {
        asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[20:21]" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 13) {
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[k]) : "v"(acc[(k + 1) % CH]));
      } else if constexpr (OP == 14) {
        asm volatile("v_mad_u64_u32 %0, s[60:61], %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b) : "s60", "s61");
      } else if constexpr (OP == 15) {
        switch (k) {
          case 0: asm volatile("v_add_co_u32_e64 %0, s[20:21], %0, %2\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[20:21], %1, 0, s[20:21]" : "+v"(a[k]), "+v"(h[k]) : "v"(b) : "s20", "s21"); break;
          case 1: asm volatile("v_add_co_u32_e64 %0, s[22:23], %0, %2\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[22:23], %1, 0, s[22:23]" : "+v"(a[k]), "+v"(h[k]) : "v"(b) : "s22", "s23"); break;
          case 2: asm volatile("v_add_co_u32_e64 %0, s[24:25], %0, %2\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[24:25], %1, 0, s[24:25]" : "+v"(a[k]), "+v"(h[k]) : "v"(b) : "s24", "s25"); break;
          case 3: asm volatile("v_add_co_u32_e64 %0, s[26:27], %0, %2\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[26:27], %1, 0, s[26:27]" : "+v"(a[k]), "+v"(h[k]) : "v"(b) : "s26", "s27"); break;
          case 4: asm volatile("v_add_co_u32_e64 %0, s[28:29], %0, %2\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[28:29], %1, 0, s[28:29]" : "+v"(a[k]), "+v"(h[k]) : "v"(b) : "s28", "s29"); break;
          case 5: asm volatile("v_add_co_u32_e64 %0, s[30:31], %0, %2\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[30:31], %1, 0, s[30:31]" : "+v"(a[k]), "+v"(h[k]) : "v"(b) : "s30", "s31"); break;
          case 6: asm volatile("v_add_co_u32_e64 %0, s[56:57], %0, %2\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[56:57], %1, 0, s[56:57]" : "+v"(a[k]), "+v"(h[k]) : "v"(b) : "s56", "s57"); break;
          case 7: asm volatile("v_add_co_u32_e64 %0, s[34:35], %0, %2\n\ts_nop 1\n\tv_addc_co_u32_e64 %1, s[34:35], %1, 0, s[34:35]" : "+v"(a[k]), "+v"(h[k]) : "v"(b) : "s34", "s35"); break;
        }
      } else if constexpr (OP == 16) {
        asm volatile("v_bfe_u32 %0, %0, 3, 21" : "+v"(a[k]));
      } else if constexpr (OP == 17) {
        asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 18) {
        asm volatile("v_mad_u64_u32 %0, s[60:61], %1, %2, %0" : "+v"(acc[0]) : "v"(a[k]), "v"(b) : "s60", "s61");
      } else if constexpr (OP == 19) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[0]) : "v"(b));
      } else if constexpr (OP == 20) {
        asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(a[k]) : "v"(b) : "vcc");
      } else if constexpr (OP == 21) {
        asm volatile("v_addc_co_u32_e32 %0, vcc, %0, %1, vcc" : "+v"(a[k]) : "v"(b) : "vcc");
      } else if constexpr (OP == 22) {
        asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 23) {
        asm volatile("v_lshlrev_b32_e32 %0, 3, %0" : "+v"(a[k]));
      } else if constexpr (OP == 24) {
        asm volatile("v_or_b32_e32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 25) {
        asm volatile("v_sub_u32_e32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 26) {
        asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 27) {
        asm volatile("v_subb_co_u32_e32 %0, vcc, %0, %1, vcc" : "+v"(a[k]) : "v"(b) : "vcc");
      } else if constexpr (OP == 28) {
        asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 29) {
        asm volatile("v_lshrrev_b32_e32 %0, 3, %0" : "+v"(a[k]));
      } else if constexpr (OP == 30) {
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 31) {
        // two independent mad->addc pairs interleaved so each addc_e32 reads vcc
        // one instruction after... (vcc is single: pair k's addc follows its mad
        // with pair k's independent add in between)
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_add_u32_e32 %1, %1, %3\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                     : "+v"(acc[k]), "+v"(h[k]) : "v"(a[k]), "v"(b) : "vcc");
      } else if constexpr (OP == 32) {
        if (k == 0) asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1" : : "v"(a[7]), "v"(b) : "vcc");
        asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(h[k]));
      } else if constexpr (OP == 33) {
        if (k == 0) asm volatile("v_cmp_gt_u32_e64 s[20:21], %0, %1" : : "v"(a[7]), "v"(b) : "s20", "s21");
        asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[20:21]" : "+v"(a[k]) : "v"(h[k]));
      } else if constexpr (OP == 34) {
        asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(a[k]) : "v"(h[(k + 1) % CH]));
        asm volatile("" : "+v"(h[(k + 1) % CH]));
      } else if constexpr (OP == 35) {
        asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(h[k]));
      } else if constexpr (OP == 36) {
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
      } else if constexpr (OP == 37) {
        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[0]) : "v"(b), "v"(h[k]));
      } else if constexpr (OP == 38) {
        asm volatile("v_addc_co_u32_e64 %0, s[20:21], %0, %1, s[20:21]\n\ts_nop 1" : "+v"(a[0]) : "v"(b) : "s20", "s21");
      } else if constexpr (OP == 39) {
        asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[0]));
      } else if constexpr (OP == 40) {
        asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[0]) : "v"(b), "v"(h[k]));
      } else if constexpr (OP == 41) {
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[0]) : "v"(acc[(k + 1) % CH]));
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) s ^= a[k] ^ h[k] ^ (uint32_t)acc[k] ^ (uint32_t)(acc[k] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) st[blockIdx.x] = Stamp{t0, t1, r0, r1};
}

template <int OP>
int run(int n_cu, int wps) {
  const int threads = 256, blocks = n_cu * wps;  // wps waves per SIMD (a block: one wave on each of 4 SIMDs)
  uint32_t* out; Stamp* st;
  CHECK(hipMalloc(&out, sizeof(uint32_t) * threads * blocks));
  CHECK(hipMalloc(&st, sizeof(Stamp) * blocks));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, 12345u, out, st);
  CHECK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, 12345u + r, out, st);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<Stamp> hs(blocks);
  CHECK(hipMemcpy(hs.data(), st, sizeof(Stamp) * blocks, hipMemcpyDeviceToHost));
  double clk = 0; int nc = 0;
  std::vector<double> loop;  // in-kernel shader cycles of one block's loop (s_memtime)
  for (auto& s : hs) if (s.r1 > s.r0) {
    clk += (double)(s.t1 - s.t0) / (double)(s.r1 - s.r0) * 100e6; ++nc;
    loop.push_back((double)(s.t1 - s.t0));
  }
  clk /= nc;
  std::sort(loop.begin(), loop.end());
  // SIMD cycles per wave-instruction: cycles * SIMDs / (waves * instructions)
  const double waves = (double)reps * blocks * (threads / 64);
  const double instr_per_wave = (double)ITERS * CH * NINSTR[OP];
  const double cyc = ms * 1e-3 * clk * (n_cu * 4.0) / (waves * instr_per_wave);
  // the same from the loop's own clock (no launch overhead): wps waves share a SIMD
  const double cyc_loop = loop.empty() ? 0.0 : loop[loop.size() / 2] / (instr_per_wave * wps);
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"simd_cycles_per_wave_instr\": %.2f, "
         "\"loop_cycles_per_wave_instr\": %.2f, \"instr_per_step\": %d, \"clk_ghz\": %.3f}\n",
         NAMES[OP], wps, cyc, cyc_loop, NINSTR[OP], clk * 1e-9);
  CHECK(hipFree(out)); CHECK(hipFree(st));
  return 0;
}

int main() {
  hipDeviceProp_t p; if (hipGetDeviceProperties(&p, 0) != hipSuccess) { fprintf(stderr, "no device\n"); return 1; }
  const int n_cu = p.multiProcessorCount;
  printf("# device %s CUs %d; SIMD cycles per wave64 instruction, 8 independent chains/lane (or one, the "
         "dependent rows), at 8 and at 1 wave(s) per SIMD\n", p.gcnArchName, n_cu);
  int rc = 0;
  for (int wps : {8, 1}) {
    rc |= run<0>(n_cu, wps); rc |= run<1>(n_cu, wps); rc |= run<2>(n_cu, wps); rc |= run<3>(n_cu, wps);
    rc |= run<4>(n_cu, wps); rc |= run<5>(n_cu, wps); rc |= run<6>(n_cu, wps); rc |= run<7>(n_cu, wps);
    rc |= run<8>(n_cu, wps); rc |= run<9>(n_cu, wps); rc |= run<10>(n_cu, wps); rc |= run<11>(n_cu, wps);
    rc |= run<12>(n_cu, wps); rc |= run<13>(n_cu, wps); rc |= run<14>(n_cu, wps); rc |= run<15>(n_cu, wps);
    rc |= run<16>(n_cu, wps); rc |= run<17>(n_cu, wps); rc |= run<18>(n_cu, wps); rc |= run<19>(n_cu, wps);
    rc |= run<20>(n_cu, wps); rc |= run<21>(n_cu, wps); rc |= run<22>(n_cu, wps); rc |= run<23>(n_cu, wps);
    rc |= run<24>(n_cu, wps); rc |= run<25>(n_cu, wps); rc |= run<26>(n_cu, wps); rc |= run<27>(n_cu, wps);
    rc |= run<28>(n_cu, wps); rc |= run<29>(n_cu, wps); rc |= run<30>(n_cu, wps); rc |= run<31>(n_cu, wps);
    rc |= run<32>(n_cu, wps); rc |= run<33>(n_cu, wps); rc |= run<34>(n_cu, wps); rc |= run<35>(n_cu, wps);
    rc |= run<36>(n_cu, wps); rc |= run<37>(n_cu, wps); rc |= run<38>(n_cu, wps); rc |= run<39>(n_cu, wps);
    rc |= run<40>(n_cu, wps); rc |= run<41>(n_cu, wps);
  }
  return rc;
}

