// A one-thread marker kernel that writes the 100-MHz wall clock
// (s_memrealtime, the counter the block kernel's group stamps read) into
// out[slot]: launched on a stream just before and after a call, it gives two
// (tick, rocprofv3 ns) pairs, so the block kernel's workgroup stamps can be
// placed on the kernel trace's time axis (tools/block_gap.py).
//
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/stamp_marker.hip -o tools/libstampmarker.so
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void hkv_stamp_marker_kernel(unsigned long long* out, uint32_t slot) {
  out[slot] = wall_clock64();
}

extern "C" int stamp_marker(void* out, uint32_t slot, void* stream) {
  hipLaunchKernelGGL(hkv_stamp_marker_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream,
                     (unsigned long long*)out, slot);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
