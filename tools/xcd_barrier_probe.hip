// Probe (round 4, for the inner loop's exchange): the latency of one grid barrier among G
// single-wave workgroups, per signalling method, with the workgroups spread over the XCDs (a
// plain stream) or confined to one XCD (a CU-masked stream; the kernel reports each workgroup's
// XCC_ID so the confinement is checked, not assumed).
//   mode 0: arrival = agent-scope atomic add on one counter, poll = agent-scope load (sc1) --
//           the persistent loop's current scheme
//   mode 1: arrival = a plain store of the step number into the workgroup's own 128-B flag line,
//           poll = workgroup-scope loads (sc0: L1 miss, L2 hit) of all G flags -- only coherent
//           when every workgroup shares one XCD's L2
//   mode 2: as 1 with agent-scope stores and polls (sc1)
// Placement: "plain" = G workgroups on a plain stream; "mask*" = the same on CU-masked streams;
// "stride8" = 8 G workgroups of which only blockIdx % 8 == 0 take part (the dispatcher deals
// workgroups to the XCDs round-robin, so these should share one XCD -- checked via XCC_ID).
// Every poll loop is bounded (spin limit), so a stale read ends the run with a flag, not a hang.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/xcd_barrier_probe tools/xcd_barrier_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr long SPIN_LIMIT = 2000000;

__global__ void bar_kernel(unsigned* cnt, unsigned* flags, int iters, int mode, unsigned* xcc_out,
                           unsigned long long* t_out, unsigned* err, int stride) {
  if (blockIdx.x % stride) return;
  const int G = gridDim.x / stride, g = blockIdx.x / stride, lane = threadIdx.x;
  if (lane == 0) {
    unsigned xcc;  // (only the taking-part workgroups record theirs)
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc_out[g] = xcc;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool bad = false;
  for (int s = 0; s < iters && !bad; ++s) {
    if (mode == 0) {
      if (lane == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)G * (unsigned)(s + 1);
      long spins = 0;
      while (true) {
        const unsigned c = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c >= target) break;
        if (++spins > SPIN_LIMIT) { bad = true; break; }
      }
    } else {
      if (lane == 0) {
        if (mode == 1) __hip_atomic_store(flags + g * 32, (unsigned)(s + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else __hip_atomic_store(flags + g * 32, (unsigned)(s + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      long spins = 0;
      while (true) {
        unsigned v = 0xffffffffu;
        if (lane < G)
          v = mode == 1 ? __hip_atomic_load(flags + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                        : __hip_atomic_load(flags + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool done = __builtin_amdgcn_read_exec() == 0 ? true : (__ballot(v < (unsigned)(s + 1)) == 0);
        if (done) break;
        if (++spins > SPIN_LIMIT) { bad = true; break; }
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    t_out[g] = t1 - t0;
    if (bad) atomicAdd(err, 1u);
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  unsigned *cnt, *flags, *xcc, *err;
  unsigned long long* tt;
  CK(hipMalloc(&cnt, 256));
  CK(hipMalloc(&flags, 64 * 128));
  CK(hipMalloc(&xcc, 64 * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&tt, 64 * 8));
  // streams: plain; masks A = CU bits 0..31, B = bits 8k (k = 0..31)
  std::vector<hipStream_t> st(3);
  CK(hipStreamCreate(&st[0]));
  const int words = (ncu + 31) / 32;
  std::vector<unsigned> mA(words, 0), mB(words, 0);
  for (int i = 0; i < 32 && i < ncu; ++i) mA[i / 32] |= 1u << (i % 32);
  for (int k = 0; k < 32 && 8 * k < ncu; ++k) mB[(8 * k) / 32] |= 1u << ((8 * k) % 32);
  CK(hipExtStreamCreateWithCUMask(&st[1], words, mA.data()));
  CK(hipExtStreamCreateWithCUMask(&st[2], words, mB.data()));
  const char* sn[4] = {"plain", "maskA_bits0-31", "maskB_bits8k", "stride8"};
  printf("{\"cus\": %d, \"iters\": %d, \"runs\": [\n", ncu, iters);
  bool first = true;
  for (int si = 0; si < 4; ++si)
    for (int G : {16, 30, 32})
      for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
          const int stride = si == 3 ? 8 : 1;
          hipStream_t s = st[si == 3 ? 0 : si];
          CK(hipMemsetAsync(cnt, 0, 256, s));
          CK(hipMemsetAsync(flags, 0, 64 * 128, s));
          CK(hipMemsetAsync(err, 0, 4, s));
          hipLaunchKernelGGL(bar_kernel, dim3(G * stride), dim3(64), 0, s, cnt, flags, iters, mode, xcc, tt, err, stride);
          CK(hipGetLastError());
          CK(hipStreamSynchronize(s));
          if (rep == 0) continue;  // warm-up
          unsigned hx[64], he;
          unsigned long long ht[64];
          CK(hipMemcpy(hx, xcc, G * 4, hipMemcpyDeviceToHost));
          CK(hipMemcpy(ht, tt, G * 8, hipMemcpyDeviceToHost));
          CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
          unsigned long long tmax = 0;
          int nx[16] = {0};
          for (int i = 0; i < G; ++i) {
            tmax = ht[i] > tmax ? ht[i] : tmax;
            nx[hx[i] & 15]++;
          }
          int xcds = 0;
          for (int i = 0; i < 16; ++i) xcds += nx[i] > 0;
          // s_memrealtime: 100 MHz
          printf("%s{\"stream\": \"%s\", \"G\": %d, \"mode\": %d, \"xcds\": %d, \"stale_wgs\": %u, \"us_per_barrier\": %.3f}",
                 first ? "" : ",\n", sn[si], G, mode, xcds, he, tmax * 0.01 / iters);
          first = false;
          fflush(stdout);
        }
      }
  printf("\n]}\n");
  return 0;
}
