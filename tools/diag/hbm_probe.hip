// Diagnostic: streaming-read bandwidth of a buffer (sum of uint4 words), to compare with the
// filter GEMM's effective HBM rate on the same data.
#include <hip/hip_runtime.h>
#include <cstdint>
__global__ __launch_bounds__(256) void stream_read(const uint4* __restrict__ p, int64_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
extern "C" int hbm_probe(const void* p, int64_t bytes, void* out, int grid, void* stream) {
    stream_read<<<grid, 256, 0, (hipStream_t)stream>>>((const uint4*)p, bytes / 16, (uint32_t*)out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
