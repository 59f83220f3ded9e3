// Same-address atomic throughput on gfx950 (diagnostic for the work-queue design):
// W one-wave workgroups each do R atomicAdd (lane 0 only) on ONE counter; prints ns per atomic.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void bump(unsigned *ctr, int reps, unsigned *sink) {
    unsigned acc = 0;
    for (int r = 0; r < reps; ++r)
        if (threadIdx.x == 0) acc += atomicAdd(ctr, 1u);
    if (threadIdx.x == 0 && acc == 0xffffffffu) sink[0] = acc;
}

int main() {
    unsigned *ctr, *sink;
    hipMalloc(&ctr, 256);
    hipMalloc(&sink, 256);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int waves : {256, 1024, 4096}) {
        for (int reps : {1, 4}) {
            hipMemset(ctr, 0, 4);
            hipLaunchKernelGGL(bump, dim3(waves), dim3(64), 0, 0, ctr, reps, sink);
            hipDeviceSynchronize();
            hipEventRecord(a);
            for (int it = 0; it < 10; ++it) hipLaunchKernelGGL(bump, dim3(waves), dim3(64), 0, 0, ctr, reps, sink);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double per = ms * 1e6 / 10 / (double(waves) * reps);
            printf("{\"waves\": %d, \"reps\": %d, \"us_per_launch\": %.2f, \"ns_per_atomic\": %.3f}\n", waves, reps,
                   ms * 1e3 / 10, per);
        }
    }
    return 0;
}
