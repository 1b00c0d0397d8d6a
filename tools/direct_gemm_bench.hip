// Feasibility probe for a barrier-free conv main loop: one wave per workgroup, a
// 64 x 64 output tile, bf16x3 operands in the S-layout (128-B lines: 32 hi | 32 lo bf16 per
// 32-channel block) loaded STRAIGHT into MFMA operand registers (per fragment of 16 rows: the hi
// and lo halves of each line as two adjacent 16-B loads), K tiles double-buffered in registers,
// no LDS and no barrier; split-K over blockIdx.z (fp32 partial stores).  A 1x1-conv GEMM:
// C[M][N] = A[M][K] . B[N][K]^T.  Prints us per call and TFLOP/s for the layer3 / layer4 shapes,
// to compare with the LDS-DMA kernel's per-launch times (profiles/r3/final/conv_table.md).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/direct_gemm_bench.hip -o tools/direct_gemm_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct Frags {
  bf16x8 ah[4], al[4], bh[4], bl[4];
};

template <int MINW>
__global__ __launch_bounds__(64, MINW) void direct_gemm(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                         int M, int N, int K, int ksplit, float* __restrict__ C) {
  const int lane = threadIdx.x;
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64, ks = blockIdx.z;
  const int KT = K / 32;                       // 32-channel blocks = K tiles
  const int kt_per = (KT + ksplit - 1) / ksplit;
  const int kt0 = ks * kt_per, kt1 = min(KT, kt0 + kt_per);
  const int r = lane & 15, ch = (lane >> 4) * 8;  // fragment row, channel chunk (8 bf16 = 16 B)
  const long lineA = (long)KT * 64;              // bf16 per A / B row (K/32 lines of 64 bf16)
  const __bf16* ap[4];
  const __bf16* bp[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ap[i] = A + (long)min(m0 + 16 * i + r, M - 1) * lineA + ch;
    bp[i] = B + (long)(n0 + 16 * i + r) * lineA + ch;
  }
  auto load = [&](Frags& F, int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      F.ah[i] = *(const bf16x8*)(ap[i] + kt * 64);
      F.al[i] = *(const bf16x8*)(ap[i] + kt * 64 + 32);
      F.bh[i] = *(const bf16x8*)(bp[i] + kt * 64);
      F.bl[i] = *(const bf16x8*)(bp[i] + kt * 64 + 32);
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfmas = [&](const Frags& F) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F.al[i], F.bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F.ah[i], F.bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F.ah[i], F.bh[j], acc[i][j], 0, 0, 0);
      }
  };
  Frags F0, F1;
  if (kt0 < kt1) load(F0, kt0);
  for (int kt = kt0; kt < kt1; kt += 2) {
    if (kt + 1 < kt1) load(F1, kt + 1);
    mfmas(F0);
    if (kt + 1 < kt1) {
      if (kt + 2 < kt1) load(F0, kt + 2);
      mfmas(F1);
    }
  }
  // D of 16x16x32: lane holds rows 4 (lane >> 4) + q, column lane & 15
  float* cp = C + (long)ks * M * N;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = m0 + 16 * i + 4 * (lane >> 4) + q;
      if (m < M)
#pragma unroll
        for (int j = 0; j < 4; ++j) cp[(long)m * N + n0 + 16 * j + r] = acc[i][j][q];
    }
}

static float bf(float x) { return x; }

int main() {
  struct Shape {
    const char* name;
    int M, N, K;
  } shapes[] = {{"l3 1024->256 1x1 (LDS-DMA kernel 24.6-25.6 us)", 7200, 256, 1024},
                {"l3 256->1024 1x1 (25.0 us)", 7200, 1024, 256},
                {"l4 512->2048 1x1 (58-65 us)", 7200, 2048, 512},
                {"l4 2048->512 1x1 (56-57 us)", 7200, 512, 2048},
                {"l3 3x3 256->256 as K=2304 (42 us)", 7200, 256, 2304},
                {"l4 3x3 512->512 as K=4608 (93-96 us)", 7200, 512, 4608}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (const Shape& s : shapes) {
    const size_t na = (size_t)s.M * s.K * 2, nb = (size_t)s.N * s.K * 2;  // bf16 elements (hi + lo)
    __bf16 *A, *B;
    float* C;
    hipMalloc(&A, na * 2);
    hipMalloc(&B, nb * 2);
    hipMalloc(&C, (size_t)8 * s.M * s.N * 4);
    hipMemset(A, 0, na * 2);
    hipMemset(B, 0, nb * 2);
    for (int ksplit : {1, 2, 4}) {
      dim3 grid((s.M + 63) / 64, s.N / 64, ksplit);
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((direct_gemm<2>), grid, dim3(64), 0, 0, A, B, s.M, s.N, s.K, ksplit, C);
      hipDeviceSynchronize();
      float best = 1e30f;
      for (int rep = 0; rep < 10; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((direct_gemm<2>), grid, dim3(64), 0, 0, A, B, s.M, s.N, s.K, ksplit, C);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double fl = 2.0 * s.M * s.N * s.K;
      printf("%-46s split %d waves %6u: %8.1f us  %6.1f TF (bf16x3 roof 838.9)\n", s.name, ksplit,
             grid.x * grid.y * grid.z, best * 1e3, fl / (best * 1e-3) / 1e12);
    }
    hipFree(A);
    hipFree(B);
    hipFree(C);
  }
  hipError_t e = hipGetLastError();
  printf("status %s\n", hipGetErrorString(e));
  (void)bf;
  return e == hipSuccess ? 0 : 1;
}
