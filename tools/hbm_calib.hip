// Diagnostic: calibrate rocprofv3 FETCH_SIZE for the solve kernel's access
// width (8-byte, lane-consecutive global loads) on gfx950. Reads a known byte
// count once; compare FETCH_SIZE * 1024 with it (MI355X_MICROARCH.md: FETCH_SIZE
// is calibrated only for 16-B-per-lane streams, where it reads half).
//   hipcc --offload-arch=gfx950 -O3 -o build/hbm_calib tools/hbm_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT -- ./build/hbm_calib
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void read8(const double *__restrict__ x, size_t n, double *out) {
    double acc = 0.0;
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        acc += x[i];
    if (acc == 12345.678) out[0] = acc;  // keep the loads
}

__global__ void read16(const double2 *__restrict__ x, size_t n, double *out) {
    double acc = 0.0;
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        acc += x[i].x + x[i].y;
    if (acc == 12345.678) out[0] = acc;
}

int main() {
    const size_t bytes = size_t(1) << 30;
    double *x, *out;
    if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
    (void)hipMemset(x, 0, bytes);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(read8, dim3(2048), dim3(256), 0, 0, x, bytes / 8, out);
        hipLaunchKernelGGL(read16, dim3(2048), dim3(256), 0, 0, reinterpret_cast<double2 *>(x), bytes / 16, out);
    }
    (void)hipDeviceSynchronize();
    std::printf("{\"bytes_read_per_launch\": %zu}\n", bytes);
    (void)hipFree(x);
    (void)hipFree(out);
    return 0;
}
