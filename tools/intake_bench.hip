// Per-CU operand intake from the XCD's L2, the limit DESIGN.md §3 puts under the small convs:
// how fast can one workgroup per CU (or two) pull a GEMM operand stream of 128-B rows into
//   mode 0: LDS by LDS-DMA (global_load_lds_dwordx4, the conv kernels' form), a DEPTH-slot ring,
//           one counted vmcnt wait + barrier per 32-KB tile;
//   mode 1: VGPRs by global_load_dwordx4 (no LDS), two register sets (tile t+1 in flight while
//           tile t is summed);
//   mode 2: VGPRs by global_load_dwordx4, then ds_write_b128 into a DEPTH-slot LDS ring, one
//           barrier per tile (register-staged operand loads);
//   mode 3: hybrid (round 3): half of each tile's pieces by LDS-DMA (issued DEPTH-1 tiles ahead),
//           half by global_load_dwordx4 one tile ahead + ds_write_b128 into the same ring slot.
//   mode 5: LDS-DMA with NO workgroup barrier: each wave streams its own pieces into its own part
//           of the DEPTH-slot ring and reads only what it loaded (vmcnt wait only) -- the DMA
//           path's own rate, to tell whether the per-tile barrier or the path sets the ceiling.
//   mode 6: mode 0's shared tile (each wave loads 1/NW of it and reads another wave's piece) with
//           the per-tile workgroup barrier replaced by LDS counters: FULL[slot] (each wave adds 1
//           once its own pieces have landed; readers wait for NW per use of the slot) and
//           FREE[slot] (each wave adds 1 after reading; a refill waits for NW per earlier use).
// Every workgroup streams its own rotation of a shared 2 MB row set (L2-resident, like the
// weight / activation rows of a conv tile).  Prints GB/s per CU for each form.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/intake_bench.hip -o tools/intake_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define LDSP __attribute__((address_space(3)))
#define GLBP __attribute__((address_space(1)))

constexpr int TILE = 32768;             // bytes per tile (256 rows x 128 B)
constexpr int PIECES = TILE / 1024;     // wave-instructions of 1 KB per tile

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int MODE, int NW, int DEPTH>
__global__ __launch_bounds__(NW * 64) void intake(const char* __restrict__ buf, int nrows, int iters, float* sink) {
  constexpr int PW = PIECES / NW;  // pieces per wave per tile
  __shared__ __attribute__((aligned(16))) char lds[MODE == 1 ? 16 : DEPTH * TILE];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int rsub = lane >> 3, csub = (lane & 7) * 16;
  const int base = (blockIdx.x * 977) % nrows;
  auto src_of = [&](int t, int j) {
    const int row = (base + t * 256 + (wv * PW + j) * 8 + rsub) % nrows;
    return buf + (long)row * 128 + csub;
  };
  float acc = 0.f;
  if (MODE == 0) {
    for (int t = 0; t < DEPTH - 1 && t < iters; ++t)
#pragma unroll
      for (int j = 0; j < PW; ++j)
        __builtin_amdgcn_global_load_lds((const GLBP void*)src_of(t, j),
                                         (LDSP void*)(lds + (t % DEPTH) * TILE + (wv * PW + j) * 1024), 16, 0, 0);
    for (int t = 0; t < iters; ++t) {
      if (t + DEPTH - 1 < iters)
        wait_vm<PW * (DEPTH - 2)>();
      else
        wait_vm<0>();
      __syncthreads();
      if (t + DEPTH - 1 < iters) {
        const int tt = t + DEPTH - 1;
#pragma unroll
        for (int j = 0; j < PW; ++j)
          __builtin_amdgcn_global_load_lds((const GLBP void*)src_of(tt, j),
                                           (LDSP void*)(lds + (tt % DEPTH) * TILE + (wv * PW + j) * 1024), 16, 0, 0);
      }
      acc += *(const float*)(lds + (t % DEPTH) * TILE + threadIdx.x * 16);
    }
  } else if (MODE == 1) {
    f32x4 a[PW], b[PW];
#pragma unroll
    for (int j = 0; j < PW; ++j) a[j] = *(const f32x4*)src_of(0, j);
    for (int t = 0; t < iters; t += 2) {
#pragma unroll
      for (int j = 0; j < PW; ++j) b[j] = *(const f32x4*)src_of(t + 1, j);
#pragma unroll
      for (int j = 0; j < PW; ++j) acc += a[j][0] + a[j][3];
#pragma unroll
      for (int j = 0; j < PW; ++j) a[j] = *(const f32x4*)src_of(t + 2, j);
#pragma unroll
      for (int j = 0; j < PW; ++j) acc += b[j][0] + b[j][3];
    }
  } else if (MODE == 3) {
    constexpr int PD = PW / 2;  // pieces per wave by LDS-DMA; the other PW - PD through registers
    auto dma = [&](int t) {
#pragma unroll
      for (int j = 0; j < PD; ++j)
        __builtin_amdgcn_global_load_lds((const GLBP void*)src_of(t, j),
                                         (LDSP void*)(lds + (t % DEPTH) * TILE + (wv * PW + j) * 1024), 16, 0, 0);
    };
    f32x4 r[PW - PD];
    for (int t = 0; t < DEPTH - 1 && t < iters; ++t) dma(t);
#pragma unroll
    for (int j = 0; j < PW - PD; ++j) r[j] = *(const f32x4*)src_of(0, PD + j);
    for (int t = 0; t < iters; ++t) {
      // tile t's register half (loaded one step ago, BEFORE that step's DMA) lands and goes to its
      // slot; its DMA half was issued DEPTH-1 steps ago: only the youngest DMA may stay in flight
      if (DEPTH >= 3 && t + DEPTH - 2 < iters && t > 0)
        wait_vm<PD>();
      else
        wait_vm<0>();
      char* slot = lds + (t % DEPTH) * TILE;
#pragma unroll
      for (int j = 0; j < PW - PD; ++j) *(f32x4*)(slot + (wv * PW + PD + j) * 1024 + lane * 16) = r[j];
      __syncthreads();
      if (t + 1 < iters) {
#pragma unroll
        for (int j = 0; j < PW - PD; ++j) r[j] = *(const f32x4*)src_of(t + 1, PD + j);
      }
      if (t + DEPTH - 1 < iters) dma(t + DEPTH - 1);
      acc += *(const float*)(lds + (t % DEPTH) * TILE + threadIdx.x * 16);
    }
  } else if (MODE == 5) {
    for (int t = 0; t < DEPTH - 1 && t < iters; ++t)
#pragma unroll
      for (int j = 0; j < PW; ++j)
        __builtin_amdgcn_global_load_lds((const GLBP void*)src_of(t, j),
                                         (LDSP void*)(lds + (t % DEPTH) * TILE + (wv * PW + j) * 1024), 16, 0, 0);
    for (int t = 0; t < iters; ++t) {
      if (t + DEPTH - 1 < iters)
        wait_vm<PW * (DEPTH - 2)>();
      else
        wait_vm<0>();
      // this wave's own 1-KB pieces of tile t (no other wave's data is read)
      acc += *(const float*)(lds + (t % DEPTH) * TILE + (wv * PW) * 1024 + lane * 16);
      if (t + DEPTH - 1 < iters) {
        const int tt = t + DEPTH - 1;
        // the slot being refilled was read at step t - 1 by this wave only: its ds_read has
        // returned (the add above consumed an LDS value issued after it)
#pragma unroll
        for (int j = 0; j < PW; ++j)
          __builtin_amdgcn_global_load_lds((const GLBP void*)src_of(tt, j),
                                           (LDSP void*)(lds + (tt % DEPTH) * TILE + (wv * PW + j) * 1024), 16, 0, 0);
      }
    }
  } else if (MODE == 6) {
    __shared__ int full[DEPTH], freec[DEPTH];
    if (threadIdx.x < DEPTH) {
      full[threadIdx.x] = 0;
      freec[threadIdx.x] = 0;
    }
    __syncthreads();
    volatile LDSP int* vfull = (volatile LDSP int*)full;
    volatile LDSP int* vfree = (volatile LDSP int*)freec;
    auto issue = [&](int tt) {
#pragma unroll
      for (int j = 0; j < PW; ++j)
        __builtin_amdgcn_global_load_lds((const GLBP void*)src_of(tt, j),
                                         (LDSP void*)(lds + (tt % DEPTH) * TILE + (wv * PW + j) * 1024), 16, 0, 0);
    };
    for (int t = 0; t < DEPTH - 1 && t < iters; ++t) issue(t);
    for (int t = 0; t < iters; ++t) {
      const int slot = t % DEPTH, use = t / DEPTH;
      if (t + DEPTH - 1 < iters)
        wait_vm<PW * (DEPTH - 2)>();
      else
        wait_vm<0>();
      if (lane == 0) __hip_atomic_fetch_add(&full[slot], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      // refill the slot tile t-1 used once every wave has read it
      if (t + DEPTH - 1 < iters) {
        const int tt = t + DEPTH - 1, s2 = tt % DEPTH, prior = tt / DEPTH;
        while (vfree[s2] < NW * prior) __builtin_amdgcn_s_sleep(0);
        issue(tt);
      }
      while (vfull[slot] < NW * (use + 1)) __builtin_amdgcn_s_sleep(0);
      acc += *(const float*)(lds + slot * TILE + (((wv + 1) % NW) * PW) * 1024 + lane * 16);
      // the read above has returned (acc consumed it) before this wave releases the slot
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(&freec[slot], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  } else if (MODE == 4) {
    // half of each tile by LDS-DMA (DEPTH-slot ring), half straight into registers (two register
    // sets, never written to LDS: an operand consumed from VGPRs, as a wave-private MFMA operand)
    constexpr int PD = PW / 2, PR = PW - PD;
    auto dma = [&](int t) {
#pragma unroll
      for (int j = 0; j < PD; ++j)
        __builtin_amdgcn_global_load_lds((const GLBP void*)src_of(t, j),
                                         (LDSP void*)(lds + (t % DEPTH) * TILE + (wv * PW + j) * 1024), 16, 0, 0);
    };
    f32x4 r0[PR], r1[PR];
#pragma unroll
    for (int j = 0; j < PR; ++j) r0[j] = *(const f32x4*)src_of(0, PD + j);
    for (int t = 0; t < DEPTH - 1 && t < iters; ++t) dma(t);
    for (int t = 0; t < iters; t += 2) {
      // even step: r1 <- tile t+1 while r0 (tile t) is consumed; odd step the other way round
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int tt = t + half;
        if (tt >= iters) break;
        if (tt + DEPTH - 2 < iters && DEPTH >= 3)
          wait_vm<PD + PR>();  // the youngest DMA and register set may stay in flight
        else
          wait_vm<0>();
        __syncthreads();
        if (tt + 1 < iters) {
#pragma unroll
          for (int j = 0; j < PR; ++j) (half ? r0 : r1)[j] = *(const f32x4*)src_of(tt + 1, PD + j);
        }
        if (tt + DEPTH - 1 < iters) dma(tt + DEPTH - 1);
#pragma unroll
        for (int j = 0; j < PR; ++j) acc += (half ? r1 : r0)[j][0] + (half ? r1 : r0)[j][3];
        acc += *(const float*)(lds + (tt % DEPTH) * TILE + threadIdx.x * 16);
      }
    }
  } else {
    f32x4 a[PW];
#pragma unroll
    for (int j = 0; j < PW; ++j) a[j] = *(const f32x4*)src_of(0, j);
    for (int t = 0; t < iters; ++t) {
      char* slot = lds + (t % DEPTH) * TILE;
#pragma unroll
      for (int j = 0; j < PW; ++j) *(f32x4*)(slot + (wv * PW + j) * 1024 + lane * 16) = a[j];
      if (t + 1 < iters) {
#pragma unroll
        for (int j = 0; j < PW; ++j) a[j] = *(const f32x4*)src_of(t + 1, j);
      }
      __syncthreads();
      acc += *(const float*)(lds + (t % DEPTH) * TILE + ((threadIdx.x * 16 + 4096) % TILE));
    }
  }
  if (acc == 12345.678f) sink[blockIdx.x] = acc;
}

template <int MODE, int NW, int DEPTH>
static void run(const char* buf, int nrows, float* sink, int grid, const char* name) {
  const int iters = 400;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((intake<MODE, NW, DEPTH>), dim3(grid), dim3(NW * 64), 0, 0, buf, nrows, iters, sink);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((intake<MODE, NW, DEPTH>), dim3(grid), dim3(NW * 64), 0, 0, buf, nrows, iters, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double bytes = (double)grid * iters * TILE;
  printf("%-44s grid %4d: %8.1f us  %7.1f GB/s per CU  %6.2f TB/s chip\n", name, grid, best * 1e3,
         bytes / (best * 1e-3) / 1e9 / 256.0, bytes / (best * 1e-3) / 1e12);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  const int nrows = 16384;  // 2 MB of 128-B rows
  char* buf;
  float* sink;
  hipMalloc(&buf, (size_t)nrows * 128);
  hipMalloc(&sink, 4096 * sizeof(float));
  hipMemset(buf, 0, (size_t)nrows * 128);
  for (int grid : {256, 512}) {
    run<0, 4, 3>(buf, nrows, sink, grid, "lds-dma  4 waves ring 3");
    run<0, 4, 4>(buf, nrows, sink, grid, "lds-dma  4 waves ring 4");
    run<0, 8, 3>(buf, nrows, sink, grid, "lds-dma  8 waves ring 3");
    run<1, 4, 2>(buf, nrows, sink, grid, "regs     4 waves (2 sets)");
    run<1, 8, 2>(buf, nrows, sink, grid, "regs     8 waves (2 sets)");
    run<1, 16, 2>(buf, nrows, sink, grid, "regs    16 waves (2 sets)");
    run<2, 4, 2>(buf, nrows, sink, grid, "regs+ds_write 4 waves ring 2");
    run<2, 8, 2>(buf, nrows, sink, grid, "regs+ds_write 8 waves ring 2");
    run<3, 4, 3>(buf, nrows, sink, grid, "hybrid dma+regs 4 waves ring 3");
    run<3, 8, 3>(buf, nrows, sink, grid, "hybrid dma+regs 8 waves ring 3");
    run<3, 4, 2>(buf, nrows, sink, grid, "hybrid dma+regs 4 waves ring 2");
    run<4, 4, 3>(buf, nrows, sink, grid, "dma half + direct-regs half 4w ring 3");
    run<4, 8, 3>(buf, nrows, sink, grid, "dma half + direct-regs half 8w ring 3");
    run<4, 4, 2>(buf, nrows, sink, grid, "dma half + direct-regs half 4w ring 2");
    run<5, 4, 3>(buf, nrows, sink, grid, "lds-dma no barrier 4 waves ring 3");
    run<5, 8, 3>(buf, nrows, sink, grid, "lds-dma no barrier 8 waves ring 3");
    run<5, 4, 4>(buf, nrows, sink, grid, "lds-dma no barrier 4 waves ring 4");
    run<5, 16, 2>(buf, nrows, sink, grid, "lds-dma no barrier 16 waves ring 2");
    run<6, 4, 3>(buf, nrows, sink, grid, "lds-dma FULL/FREE 4 waves ring 3");
    run<6, 8, 3>(buf, nrows, sink, grid, "lds-dma FULL/FREE 8 waves ring 3");
    run<6, 4, 4>(buf, nrows, sink, grid, "lds-dma FULL/FREE 4 waves ring 4");
    run<6, 8, 4>(buf, nrows, sink, grid, "lds-dma FULL/FREE 8 waves ring 4");
  }
  hipError_t e = hipGetLastError();
  printf("status %s\n", hipGetErrorString(e));
  return e == hipSuccess ? 0 : 1;
}
