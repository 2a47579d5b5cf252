// FETCH_SIZE calibration probe: read a 1.08 GB fp32 plane ([32 utterances][32
// channels][264704 samples], the HiFiGAN-v1 stage-4 plane, 4x the Infinity Cache) exactly once
// with three access patterns and compare rocprofv3's FETCH_SIZE with the byte count:
//   x4     16 B per lane, coalesced (the pattern MI355X_MICROARCH.md calibrates: FETCH = 1/2 bytes)
//   dword  4 B per lane, 256 contiguous bytes per wave-instruction
//   stage  the pair / block / split staging lane map (RES_STAGE_8R): lane u of a 256-thread
//          workgroup reads time r = (u >> 5) * 8 + (u & 7) of channel 4 q + j, q = quad_pos((u >> 3) & 3),
//          j = 0..3: each wave-instruction reads 4 rows x 64 contiguous bytes, the 4 waves of a
//          workgroup complete 256-byte rows (64 samples x 16 channels per workgroup)
// usage: probe_fetch [reps]   (kernel names probe_x4 / probe_dword / probe_stage in the trace)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

constexpr int B = 32, C = 32, T = 264704;  // T % 64 == 0
constexpr size_t N = (size_t)B * C * T;

__global__ __launch_bounds__(256) void probe_x4(const float4* __restrict__ x, float* out, size_t n4) {
  float s = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void probe_dword(const float* __restrict__ x, float* out, size_t n) {
  float s = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += x[i];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

__device__ __forceinline__ int quad_pos(int q) { return q == 1 ? 2 : (q == 2 ? 1 : q); }

__global__ __launch_bounds__(256) void probe_stage(const float* __restrict__ x, float* out) {
  const int u = threadIdx.x;
  const int t0 = blockIdx.x * 64, g = blockIdx.y, b = blockIdx.z;
  const int r = (u >> 5) * 8 + (u & 7);
  const int q = quad_pos((u >> 3) & 3);
  const float* base = x + ((size_t)b * C + 16 * g + 4 * q) * T + t0 + r;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += base[(size_t)j * T];
  if (s == 1234.5f) out[u] = s;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
  float* x;
  float* out;
  CHECK(hipMalloc(&x, N * sizeof(float)));
  CHECK(hipMalloc(&out, 256 * sizeof(float)));
  CHECK(hipMemset(x, 0, N * sizeof(float)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int k = 0; k < 3; ++k) {
    for (int rep = 0; rep < reps; ++rep) {
      CHECK(hipEventRecord(e0));
      if (k == 0) hipLaunchKernelGGL(probe_x4, dim3(8192), dim3(256), 0, 0, (const float4*)x, out, N / 4);
      if (k == 1) hipLaunchKernelGGL(probe_dword, dim3(8192), dim3(256), 0, 0, x, out, N);
      if (k == 2) hipLaunchKernelGGL(probe_stage, dim3(T / 64, C / 16, B), dim3(256), 0, 0, x, out);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("%s rep %d: %.3f ms, %.2f TB/s (bytes %zu)\n", k == 0 ? "probe_x4" : (k == 1 ? "probe_dword" : "probe_stage"),
                  rep, ms, N * 4.0 / ms / 1e9, N * sizeof(float));
    }
  }
  CHECK(hipFree(x));
  CHECK(hipFree(out));
  return 0;
}
