// Development microbenchmark (not shipped): dependent-chain latency of the instruction patterns of the
// threshold scan on gfx950, one wave alone, shader cycles per step (s_memtime).
//   hipcc --offload-arch=gfx950 -O3 -o build/lat_micro tools/lat_micro.hip && ./build/lat_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int N = 256;

template <int R>
__device__ inline double ror16(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_mov_dpp(int(uint32_t(u)), 0x120 + R, 0xf, 0xf, true);
    const uint32_t hi = __builtin_amdgcn_mov_dpp(int(uint32_t(u >> 32)), 0x120 + R, 0xf, 0xf, true);
    return __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}
__device__ inline double vmin(double a, double b) {
    double r;
    asm volatile("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__global__ void k(double *out, unsigned long long *cyc, double seed, int mode) {
    __shared__ double lds[1024];
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) lds[i] = double((i * 7 + 3) & 1023);
    __syncthreads();
    double x = seed + lane, y = 1e-300;
    int ix = lane;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    switch (mode) {
    case 0:  // v_add_f64 chain
#pragma unroll 16
        for (int i = 0; i < N; ++i) { x = x + y; asm volatile("" : "+v"(x)); }
        break;
    case 1:  // v_mul_f64 chain
#pragma unroll 16
        for (int i = 0; i < N; ++i) { x = x * 1.0000001; asm volatile("" : "+v"(x)); }
        break;
    case 2:  // raw v_min_f64 chain
#pragma unroll 16
        for (int i = 0; i < N; ++i) x = vmin(x, y);
        break;
    case 3:  // row16 reduce step: 2 dpp movs + v_min_f64
#pragma unroll 16
        for (int i = 0; i < N; ++i) x = vmin(x, ror16<1>(x));
        break;
    case 4:  // compare + select (f64)
#pragma unroll 16
        for (int i = 0; i < N; ++i) { x = (x < y) ? y : x; asm volatile("" : "+v"(x)); }
        break;
    case 5:  // dependent ds_read_b64 (address from the previous value)
        for (int i = 0; i < N; ++i) { ix = int(lds[ix & 1023]); }
        x = ix;
        break;
    case 6:  // ds_bpermute chain
        for (int i = 0; i < N; ++i) ix = __shfl(ix, (ix + 1) & 63);
        x = ix;
        break;
    case 7:  // v_add_u32 chain
#pragma unroll 16
        for (int i = 0; i < N; ++i) { ix = ix + 3; asm volatile("" : "+v"(ix)); }
        x = ix;
        break;
    case 8: {  // ballot -> per-lane shift -> ctz (Seg<16>::lowest) feeding the next compare
        const int base = lane & ~15;
        for (int i = 0; i < N; ++i) {
            const uint64_t b = (__ballot(ix > 7) >> base) & 0xffff;
            ix = b ? __builtin_ctzll(b) : 0x7fffffff;
            ix = (ix + lane) & 15;
        }
        x = ix;
        break;
    }
    case 9:  // f64 subtract + fabs + fmax + mul + compare (the leaf convexity test) chained through a select
        for (int i = 0; i < N; ++i) {
            const double d = x - y;
            const bool c = d >= y - 1e-12 * fmax(1.0, fabs(x));
            x = c ? d + 1.0 : x;
        }
        break;
    case 10:  // readlane broadcast chain (uniform index)
        for (int i = 0; i < N; ++i) { ix = __builtin_amdgcn_readlane(ix, 5) + lane; }
        x = ix;
        break;
    case 11:  // 4-step row16 min reduction per iteration, chained
        for (int i = 0; i < N / 4; ++i) {
            x = vmin(x, ror16<8>(x));
            x = vmin(x, ror16<4>(x));
            x = vmin(x, ror16<2>(x));
            x = vmin(x, ror16<1>(x));
            x = x + 1.0;
        }
        break;
    case 12: {  // 8 independent v_add_f64 chains (issue rate), per instruction
        double a[8];
        for (int j = 0; j < 8; ++j) a[j] = x + j;
        for (int i = 0; i < N / 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) { a[j] = a[j] + y; asm volatile("" : "+v"(a[j])); }
        for (int j = 0; j < 8; ++j) x += a[j];
        break;
    }
    case 13: {  // 8 independent v_cmp_f64 -> v_cndmask pairs (issue rate), per select
        double a[8];
        for (int j = 0; j < 8; ++j) a[j] = x + j;
        for (int i = 0; i < N / 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) { a[j] = a[j] < y ? y : a[j]; asm volatile("" : "+v"(a[j])); }
        for (int j = 0; j < 8; ++j) x += a[j];
        break;
    }
    case 14: {  // 8 independent v_max_f64 (issue rate)
        double a[8];
        for (int j = 0; j < 8; ++j) a[j] = x + j;
        for (int i = 0; i < N / 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) { a[j] = vmin(a[j], y); asm volatile("" : "+v"(a[j])); }
        for (int j = 0; j < 8; ++j) x += a[j];
        break;
    }
    case 15: {  // 8 independent v_add_u32 (issue rate)
        int a[8];
        for (int j = 0; j < 8; ++j) a[j] = ix + j;
        for (int i = 0; i < N / 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) { a[j] = a[j] + 3; asm volatile("" : "+v"(a[j])); }
        for (int j = 0; j < 8; ++j) ix += a[j];
        x = ix;
        break;
    }
    case 16: {  // 8 independent v_mul_f64
        double a[8];
        for (int j = 0; j < 8; ++j) a[j] = x + j;
        for (int i = 0; i < N / 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) { a[j] = a[j] * 1.0000001; asm volatile("" : "+v"(a[j])); }
        for (int j = 0; j < 8; ++j) x += a[j];
        break;
    }
    case 17: {  // 8 independent int compare + select (u32)
        int a[8];
        for (int j = 0; j < 8; ++j) a[j] = ix + j;
        for (int i = 0; i < N / 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) { a[j] = a[j] < lane ? lane : a[j] + 1; asm volatile("" : "+v"(a[j])); }
        for (int j = 0; j < 8; ++j) ix += a[j];
        x = ix;
        break;
    }
    case 18: {  // 8 independent f64 selects on a loop-invariant mask (v_cndmask x2 only)
        double a[8];
        const bool m = lane & 1;
        for (int j = 0; j < 8; ++j) a[j] = x + j;
        for (int i = 0; i < N / 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) { a[j] = m ? a[j] : y; asm volatile("" : "+v"(a[j])); }
        for (int j = 0; j < 8; ++j) x += a[j];
        break;
    }
    case 19: {  // 8 independent v_cmp_f64 whose results are OR-ed into a mask (compare only)
        double a[8];
        for (int j = 0; j < 8; ++j) a[j] = x + j;
        bool acc = false;
        for (int i = 0; i < N / 8; ++i) {
#pragma unroll
            for (int j = 0; j < 8; ++j) { acc = acc | (a[j] < y); asm volatile("" : "+v"(a[j])); }
        }
        x = acc ? 1.0 : 2.0;
        break;
    }
    }
    asm volatile("" ::"v"(x));
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = x;
    if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
    double *out;
    unsigned long long *cyc, h;
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, sizeof(unsigned long long));
    const char *names[] = {"v_add_f64", "v_mul_f64", "v_min_f64", "dpp2+v_min_f64", "cmp+select f64", "ds_read_b64 dep",
                           "ds_bpermute", "v_add_u32", "ballot>>base+ctz", "leaf test", "readlane", "row16 reduce (per step)",
                           "v_add_f64 x8 indep", "cmp+sel f64 x8 indep", "v_min_f64 x8 indep", "v_add_u32 x8 indep",
                           "v_mul_f64 x8 indep", "cmp+sel u32 x8 indep", "sel f64 (fixed mask) x8",
                           "v_cmp_f64 x8 (or)"};
    for (int m = 0; m < 20; ++m) {
        for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 1.0, m);
        hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        printf("%-26s %7.1f cycles per step\n", names[m], double(h) / N);
    }
    return 0;
}
