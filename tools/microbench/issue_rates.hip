// Development microbenchmark (not product code): SALU / VALU issue rates per
// CU on gfx950, to tell whether the POA strip kernel's ~139 SALU per strip
// row compete for a shared scalar unit.  Each wave runs ITERS iterations of
// 8 independent instructions of one kind (or 8 SALU + 8 VALU interleaved).
// The SALU op is s_mul_i32: it leaves SCC alone (an SCC write inside asm would
// clobber the loop's compare-and-branch).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int ITERS = 20000;

__global__ void salu_k(int* out, int seed) {
  int a = seed, b = seed + 1, c = seed + 2, d = seed + 3, e = seed + 4, f = seed + 5, g = seed + 6, h = seed + 7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "s_mul_i32 %0, %0, 3\n\ts_mul_i32 %1, %1, 3\n\ts_mul_i32 %2, %2, 3\n\ts_mul_i32 %3, %3, 3\n\t"
        "s_mul_i32 %4, %4, 3\n\ts_mul_i32 %5, %5, 3\n\ts_mul_i32 %6, %6, 3\n\ts_mul_i32 %7, %7, 3"
        : "+s"(a), "+s"(b), "+s"(c), "+s"(d), "+s"(e), "+s"(f), "+s"(g), "+s"(h));
  }
  if (threadIdx.x == 0) out[blockIdx.x] = a + b + c + d + e + f + g + h;
}

__global__ void valu_k(int* out, int seed) {
  int a = seed + threadIdx.x, b = a + 1, c = a + 2, d = a + 3, e = a + 4, f = a + 5, g = a + 6, h = a + 7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_add_u32 %0, %0, 1\n\tv_add_u32 %1, %1, 1\n\tv_add_u32 %2, %2, 1\n\tv_add_u32 %3, %3, 1\n\t"
        "v_add_u32 %4, %4, 1\n\tv_add_u32 %5, %5, 1\n\tv_add_u32 %6, %6, 1\n\tv_add_u32 %7, %7, 1"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + e + f + g + h;
}

__global__ void mix_k(int* out, int seed) {
  int a = seed, b = seed + 1, c = seed + 2, d = seed + 3, e = seed + 4, f = seed + 5, g = seed + 6, h = seed + 7;
  int va = seed + threadIdx.x, vb = va + 1, vc = va + 2, vd = va + 3, ve = va + 4, vf = va + 5, vg = va + 6, vh = va + 7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "s_mul_i32 %0, %0, 3\n\tv_add_u32 %8, %8, 1\n\ts_mul_i32 %1, %1, 3\n\tv_add_u32 %9, %9, 1\n\t"
        "s_mul_i32 %2, %2, 3\n\tv_add_u32 %10, %10, 1\n\ts_mul_i32 %3, %3, 3\n\tv_add_u32 %11, %11, 1\n\t"
        "s_mul_i32 %4, %4, 3\n\tv_add_u32 %12, %12, 1\n\ts_mul_i32 %5, %5, 3\n\tv_add_u32 %13, %13, 1\n\t"
        "s_mul_i32 %6, %6, 3\n\tv_add_u32 %14, %14, 1\n\ts_mul_i32 %7, %7, 3\n\tv_add_u32 %15, %15, 1"
        : "+s"(a), "+s"(b), "+s"(c), "+s"(d), "+s"(e), "+s"(f), "+s"(g), "+s"(h), "+v"(va), "+v"(vb), "+v"(vc),
          "+v"(vd), "+v"(ve), "+v"(vf), "+v"(vg), "+v"(vh));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + e + f + g + h + va + vb + vc + vd + ve + vf + vg + vh;
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  int* out;
  (void)hipMalloc(&out, 64ull * 1024 * 1024);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[3] = {"salu", "valu", "mix"};
  for (int kind = 0; kind < 3; ++kind) {
    for (int wpc : {1, 4, 8, 16, 24}) {  // waves per CU (one 64-thread block = one wave)
      const int blocks = cus * wpc;
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0, 0);
        if (kind == 0) hipLaunchKernelGGL(salu_k, dim3(blocks), dim3(64), 0, 0, out, rep);
        if (kind == 1) hipLaunchKernelGGL(valu_k, dim3(blocks), dim3(64), 0, 0, out, rep);
        if (kind == 2) hipLaunchKernelGGL(mix_k, dim3(blocks), dim3(64), 0, 0, out, rep);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double insts = (kind == 2 ? 16.0 : 8.0) * ITERS * wpc;  // per CU (wave-instructions)
        const double ghz = 2.4;  // nominal; per-CU rates below are per nominal cycle
        if (rep == 1)
          std::fflush(stdout);
          std::printf("%s waves/CU %2d: %.3f ms, %.3f wave-instr per CU-cycle (%.3f per SIMD-cycle)\n", names[kind],
                      wpc, ms, insts / (ms * 1e-3 * ghz * 1e9), insts / (ms * 1e-3 * ghz * 1e9) / 4);
      }
    }
  }
  return 0;
}
