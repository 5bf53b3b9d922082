// hkv_internal.h — declarations shared between the kernel TU and the C-ABI TU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HKV_MODE_LIBSECP 0u
#define HKV_MODE_HASKOIN 1u

// debug/known-answer ops (hkv_debug_op in include/hkv.h)
enum {
  HKV_DBG_FE_MUL = 1,
  HKV_DBG_FE_SQR = 2,
  HKV_DBG_FE_ADD = 3,
  HKV_DBG_FE_SUB = 4,
  HKV_DBG_FE_INV = 5,
  HKV_DBG_FE_SQRT = 6,
  HKV_DBG_SC_MUL = 7,
  HKV_DBG_SC_INV = 8,
  HKV_DBG_GLV = 9,
  HKV_DBG_ECMULT_G = 10,
  HKV_DBG_MUL512 = 11,
  HKV_DBG_SQR512 = 12,
};

namespace hkv {
hipError_t launch_prologue(const void* recs, uint32_t n, uint32_t n_pad, uint32_t mode, uint32_t* im,
                           hipStream_t st);
hipError_t launch_ecmult(const uint32_t* im, uint32_t n, uint32_t n_pad, const uint32_t* gtab, uint32_t* qs,
                         uint32_t grid, uint32_t* bits, hipStream_t st);
hipError_t launch_gtable(uint32_t* gtab, hipStream_t st);
hipError_t launch_gen_pool(uint64_t seed, uint32_t npool, uint32_t* pool, hipStream_t st);
hipError_t launch_gen_records(uint64_t seed, uint32_t n, const uint32_t* pool, uint32_t npool,
                              uint32_t unc_permille, void* recs, hipStream_t st);
hipError_t launch_debug(uint32_t op, uint32_t n, const uint32_t* a, const uint32_t* b, uint32_t* out,
                        hipStream_t st);
hipError_t ecmult_max_blocks_per_cu(int* out);
}  // namespace hkv
