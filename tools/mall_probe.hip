// Infinity-Cache (MALL) probe: effective bandwidth of a streaming write followed by a streaming read
// of the same buffer, as a function of the buffer size.  Decides whether a chunked step schedule
// (activations written and re-read while they still sit in the 256 MiB die-level cache) can beat
// the HBM floor of writing every saved activation out and reading it back.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/mall_probe tools/mall_probe.hip && tools/mall_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_write(uint4* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4(seed, (unsigned)i, seed ^ (unsigned)i, 7u);
}

__global__ void k_read(const uint4* p, size_t n, unsigned* out) {
    unsigned s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = p[i];
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x12345678u) out[0] = s;  // keeps the loads alive
}

int main() {
    const size_t sizes_mb[] = {32, 64, 128, 192, 256, 384, 512, 1024, 4096};
    const size_t max_b = 4096ull << 20;
    uint4* buf;
    unsigned* out;
    CK(hipMalloc(&buf, max_b));
    CK(hipMalloc(&out, 4));
    hipEvent_t a, b, c;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreate(&c));
    const int grid = 256 * 8, block = 256;
    printf("size_MB  write_GBps  read_GBps  (mean of the last 10 of 14 write->read pairs)\n");
    for (size_t mb : sizes_mb) {
        const size_t n = (mb << 20) / sizeof(uint4);
        double tw = 0, tr = 0;
        for (int it = 0; it < 14; ++it) {
            CK(hipEventRecord(a, 0));
            hipLaunchKernelGGL(k_write, dim3(grid), dim3(block), 0, 0, buf, n, (unsigned)it);
            CK(hipEventRecord(b, 0));
            hipLaunchKernelGGL(k_read, dim3(grid), dim3(block), 0, 0, buf, n, out);
            CK(hipEventRecord(c, 0));
            CK(hipEventSynchronize(c));
            float w, r;
            CK(hipEventElapsedTime(&w, a, b));
            CK(hipEventElapsedTime(&r, b, c));
            if (it >= 4) { tw += w; tr += r; }
        }
        const double bytes = (double)(mb << 20);
        printf("%7zu  %10.0f  %9.0f\n", mb, bytes / (tw / 10 * 1e-3) / 1e9, bytes / (tr / 10 * 1e-3) / 1e9);
    }
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
