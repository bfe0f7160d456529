// fetch_calib.hip — calibrates rocprofv3 FETCH_SIZE for b3_groups' access
// pattern (MI355X_MICROARCH.md §HBM: the x2 gfx950 correction is measured for
// wide coalesced 16-B/lane streams only; "other access widths are
// uncalibrated").  Every kernel reads the same 16 GiB exactly once:
//   coalesced      — a wave's 16-B loads cover 1 KiB contiguous (the guide's case)
//   lane_stream<P> — b3_groups' fast path: lane g owns bytes [8 KiB g, 8 KiB (g+1)),
//                    walked as 64-B blocks of 4 x 16-B loads, lanes of a wave
//                    8 KiB apart; P = VALU ops spent per block (0: pure stream,
//                    680: one BLAKE3 compression's worth, so lines are touched
//                    at the kernel's pace)
// The known byte count (16 GiB) divided by FETCH_SIZE (KiB x 1024) gives the
// correction factor for each shape.
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      return 1;                                                          \
    }                                                                    \
  } while (0)

constexpr uint64_t kGroup = 8192;  // bytes per lane (8 leaves of 1 KiB)

__global__ __launch_bounds__(256) void coalesced(const u32x4 *__restrict__ p, uint64_t n16,
                                                 uint32_t *__restrict__ out) {
  u32x4 acc = {0, 0, 0, 0};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += stride)
    acc ^= p[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int P>
__global__ __launch_bounds__(256) void lane_stream(const uint8_t *__restrict__ data,
                                                   uint64_t groups, uint32_t *__restrict__ out) {
  const uint64_t g = blockIdx.x * 256ull + threadIdx.x;
  if (g >= groups) return;
  const u32x4 *q = reinterpret_cast<const u32x4 *>(data + g * kGroup);
  uint32_t a0 = 0, a1 = 1, a2 = 2, a3 = 3;
#pragma unroll 2
  for (int b = 0; b < (int)(kGroup / 64); ++b, q += 4) {
    const u32x4 x0 = q[0], x1 = q[1], x2 = q[2], x3 = q[3];
    a0 ^= x0.x ^ x1.y ^ x2.z ^ x3.w;
    a1 ^= x0.y ^ x1.z ^ x2.w ^ x3.x;
    a2 ^= x0.z ^ x1.w ^ x2.x ^ x3.y;
    a3 ^= x0.w ^ x1.x ^ x2.y ^ x3.z;
#pragma unroll
    for (int k = 0; k < P / 4; ++k) {  // 4 independent rotate chains
      asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a0));
      asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a1));
      asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a2));
      asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a3));
    }
  }
  out[g] = a0 ^ a1 ^ a2 ^ a3;
}

int main(int argc, char **argv) {
  const uint64_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 16ull) << 30;
  const uint64_t groups = bytes / kGroup;
  uint8_t *d;
  uint32_t *out;
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(&out, groups * sizeof(uint32_t)));
  CHECK(hipMemset(d, 0x5a, bytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const dim3 grid((unsigned)((groups + 255) / 256));
  for (int rep = 0; rep < 3; ++rep) {
    float ms[3];
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(coalesced, dim3(256 * 32), dim3(256), 0, 0,
                       reinterpret_cast<const u32x4 *>(d), bytes / 16, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms[0], e0, e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(lane_stream<0>, grid, dim3(256), 0, 0, d, groups, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms[1], e0, e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(lane_stream<680>, grid, dim3(256), 0, 0, d, groups, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms[2], e0, e1));
    printf("{\"rep\": %d, \"bytes\": %llu, \"coalesced_ms\": %.3f, \"lane_stream0_ms\": %.3f, "
           "\"lane_stream680_ms\": %.3f}\n",
           rep, (unsigned long long)bytes, ms[0], ms[1], ms[2]);
  }
  CHECK(hipFree(d));
  CHECK(hipFree(out));
  return 0;
}
