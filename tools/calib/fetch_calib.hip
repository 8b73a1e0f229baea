// fetch_calib.hip — calibration kernels for rocprofv3's FETCH_SIZE on gfx950 (measurement tool,
// not product code).  MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of the bytes of a 16-B/lane
// streaming read; other widths are uncalibrated.  Each kernel reads a known number of bytes, once,
// from a buffer far larger than the 256 MiB Infinity Cache, in one of the access shapes the narrow
// phase uses, and writes one word per workgroup; tools/calib/fetch_calib.py runs them under
// `rocprofv3 --pmc FETCH_SIZE` and prints bytes read / (FETCH_SIZE * 1024) per shape.
#include <hip/hip_runtime.h>
#include <cstdint>

// 4 bytes per lane, fully coalesced (one 256-B wave request per instruction)
__global__ void stream4(const float* __restrict__ p, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
    if (s == 12345.f) out[blockIdx.x] = s;
}
// 16 bytes per lane, fully coalesced
__global__ void stream16(const float4* __restrict__ p, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = p[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[blockIdx.x] = s;
}
// the narrow phase's hull loads (GJK tier 0): groups of 4 lanes, each group one 32-vertex fp32
// SoA hull (384 B: x[32], y[32], z[32]), lane l of a group reading element k*4 + l of each column;
// hulls in a permuted order (a pair list over a pool)
__global__ void hulls4(const float* __restrict__ p, const uint32_t* __restrict__ perm, size_t nhull, float* out) {
    const int lane = threadIdx.x & 63, g = lane >> 2, gl = lane & 3;
    float s = 0.f;
    for (size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; w * 16 < nhull; w += (size_t)gridDim.x * (blockDim.x / 64)) {
        const size_t h = w * 16 + g;
        if (h >= nhull) continue;
        const float* q = p + (size_t)perm[h] * 96;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += q[k * 4 + gl] + q[32 + k * 4 + gl] + q[64 + k * 4 + gl];
    }
    if (s == 12345.f) out[blockIdx.x] = s;
}

extern "C" int fetch_calib_run(int shape, const void* buf, size_t bytes, const uint32_t* perm, float* out, int grid) {
    if (shape == 0) hipLaunchKernelGGL(stream4, dim3(grid), dim3(256), 0, 0, (const float*)buf, bytes / 4, out);
    else if (shape == 1) hipLaunchKernelGGL(stream16, dim3(grid), dim3(256), 0, 0, (const float4*)buf, bytes / 16, out);
    else hipLaunchKernelGGL(hulls4, dim3(grid), dim3(256), 0, 0, (const float*)buf, perm, bytes / 384, out);
    return (int)hipDeviceSynchronize();
}
