// Development microbenchmark (not shipped): host cost of one kernel launch on gfx950 / ROCm 7.2 by
// launch API, for a ~920-byte argument struct (the sweep kernel's), streams not synchronised between
// launches (the bench's situation). hipcc --offload-arch=gfx950 -O3 -o build/launch_micro tools/launch_micro.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

struct Big {
    double d[115];
    int n;
};

__global__ void k_big(Big a, int *out) {
    if (threadIdx.x == 0 && a.n < 0) out[0] = 1;
}

int main() {
    int *out;
    hipMalloc(&out, 4);
    hipStream_t s1, s2;
    hipStreamCreate(&s1);
    hipStreamCreate(&s2);
    Big a;
    memset(&a, 0, sizeof(a));
    a.n = 1;
    hipFunction_t fn;
    if (hipGetFuncBySymbol(&fn, reinterpret_cast<const void *>(k_big)) != hipSuccess) printf("hipGetFuncBySymbol failed\n");
    const int N = 2000;
    for (int G : {1, 1024}) {
    printf("grid %d x 64\n", G);
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 3; ++mode) {
            hipDeviceSynchronize();
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < N; ++i) {
                hipStream_t s = (i & 1) ? s2 : s1;
                if (mode == 0) {
                    hipLaunchKernelGGL(k_big, dim3(G), dim3(64), 0, s, a, out);
                } else if (mode == 1) {
                    void *args[] = {&a, &out};
                    hipModuleLaunchKernel(fn, G, 1, 1, 64, 1, 1, 0, s, args, nullptr);
                } else {
                    struct {
                        Big a;
                        int *out;
                    } pk{a, out};
                    size_t sz = sizeof(pk);
                    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &pk, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
                    hipModuleLaunchKernel(fn, G, 1, 1, 64, 1, 1, 0, s, nullptr, cfg);
                }
            }
            auto t1 = std::chrono::steady_clock::now();
            hipDeviceSynchronize();
            auto t2 = std::chrono::steady_clock::now();
            const char *nm[] = {"hipLaunchKernelGGL", "hipModuleLaunchKernel(args)", "hipModuleLaunchKernel(buffer)"};
            printf("%-32s enqueue %.2f us/launch, wall %.2f us/launch\n", nm[mode],
                   std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
                   std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
        }
    }
    }
    return 0;
}
