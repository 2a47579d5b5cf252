// Probe: does the raw-buffer range check include the scalar soffset on gfx950?
// Descriptor with num_records = 16 bytes over a 64-float array of known values.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* x, float* out) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, 16, 0x00020000);
  const int l = threadIdx.x;
  if (l == 0) {
    out[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 0));    // in range
    out[1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 64, 0, 0));   // voffset OOB
    out[2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 0, 64, 0));   // soffset only
    out[3] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 8, 12, 0));   // sum OOB
  }
}
int main() {
  float h[64];
  for (int i = 0; i < 64; ++i) h[i] = 100.f + i;
  float *x, *o;
  hipMalloc(&x, 256); hipMalloc(&o, 16);
  hipMemcpy(x, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, x, o);
  float r[4];
  hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
  printf("inrange=%g voffOOB=%g soffOnly=%g sumOOB=%g  (0 = range-checked; 116/103 = not)\n", r[0], r[1], r[2], r[3]);
  return 0;
}
