// HBM streaming rate vs per-lane access width on MI355X: y[i] = x[i] (+ read-only stream),
// 8 B (dwordx2) vs 16 B (dwordx4) per lane. Decides whether stencil kernels should move two
// fp64 columns per lane. Build: hipcc --offload-arch=gfx950 -O3 copy_width.hip -o copy_width
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);   \
            return 1;                                                               \
        }                                                                           \
    } while (0)

template <class V>
__global__ void __launch_bounds__(256) copy(const V* __restrict__ x, V* __restrict__ y, size_t n) {
    for (size_t i = blockIdx.x * size_t(256) + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) y[i] = x[i];
}
template <class V, bool NT>
__global__ void __launch_bounds__(256) read2(const V* __restrict__ a, const V* __restrict__ b,
                                             V* __restrict__ y, size_t n) {
    for (size_t i = blockIdx.x * size_t(256) + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
        V u = a[i], v = b[i];
        if constexpr (NT) __builtin_nontemporal_store(u + v, &y[i]);
        else y[i] = u + v;
    }
}
// the temporal-blocking sweep's byte mix: two read streams, two write streams
template <class V, bool NT>
__global__ void __launch_bounds__(256) read2write2(const V* __restrict__ a, const V* __restrict__ b,
                                                   V* __restrict__ y, V* __restrict__ z, size_t n) {
    for (size_t i = blockIdx.x * size_t(256) + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
        V u = a[i], v = b[i];
        if constexpr (NT) {
            __builtin_nontemporal_store(u + v, &y[i]);
            __builtin_nontemporal_store(u - v, &z[i]);
        } else {
            y[i] = u + v;
            z[i] = u - v;
        }
    }
}

template <class V>
int run(const char* name, size_t bytes, int blocks) {
    const size_t n = bytes / sizeof(V);
    V *a, *b, *y, *z;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&y, bytes));
    CK(hipMalloc(&z, bytes));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    static const char* names[] = {"copy", "2r1w", "2r1w-nt", "2r2w", "2r2w-nt"};
    for (int mode = 0; mode < 5; ++mode) {
        float best = 1e30f;
        for (int it = 0; it < 6; ++it) {
            CK(hipEventRecord(e0));
            if (mode == 0) hipLaunchKernelGGL(copy<V>, dim3(blocks), dim3(256), 0, 0, a, y, n);
            else if (mode == 1) hipLaunchKernelGGL((read2<V, false>), dim3(blocks), dim3(256), 0, 0, a, b, y, n);
            else if (mode == 2) hipLaunchKernelGGL((read2<V, true>), dim3(blocks), dim3(256), 0, 0, a, b, y, n);
            else if (mode == 3) hipLaunchKernelGGL((read2write2<V, false>), dim3(blocks), dim3(256), 0, 0, a, b, y, z, n);
            else hipLaunchKernelGGL((read2write2<V, true>), dim3(blocks), dim3(256), 0, 0, a, b, y, z, n);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it > 0 && ms < best) best = ms;
        }
        const double moved = double(bytes) * (mode == 0 ? 2 : (mode < 3 ? 3 : 4));
        std::printf("%-10s %-8s blocks %6d: %.3f ms  %.2f TB/s\n", name, names[mode],
                    blocks, best, moved / best / 1e9);
    }
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(y));
    CK(hipFree(z));
    return 0;
}

int main() {
    const size_t bytes = size_t(2) << 30;  // 2 GiB per array
    for (int blocks : {2048, 8192, 32768}) {
        if (run<double>("f64 x1", bytes, blocks)) return 1;
        if (run<float>("f32 x1", bytes, blocks)) return 1;
    }
    return 0;
}
