// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 per access width and pattern (MI355X_MICROARCH.md:
// "other access widths are uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Every kernel below touches a KNOWN number of distinct HBM bytes (buffers of 2 GiB, far past the 256 MiB
// Infinity Cache, each byte touched once per launch), one launch per pattern, so a --pmc pass gives
// counter / true bytes per pattern.  tools/pmc_traffic.py applies the resulting factors per kernel.
//
//   read16   float4 per lane, coalesced streaming read           (NVT rows, snapshot rows streamed)
//   read8    float2 per lane, coalesced
//   read4    int per lane, coalesced                              (column-major list reads: idx[t*N + i])
//   write16  float4 per lane, coalesced streaming store           (f_n / positions / edge vectors)
//   write4   int per lane, coalesced store                        (column-major list stores by the anchor test)
//   scat4    one 4-B store per 128-B line, every line of the buffer (a sparse column store: one row of a column)
//   rowcol4  one wave per row, lane t stores column t of that row: the requery's 64 list stores per re-anchored row,
//            for every 16th row (DENSE would be every row)
//   gath16   16-B gathers of random rows of a 2 GiB table (L2-miss granularity of a row gather)
//
// build: hipcc -O3 --offload-arch=gfx950 tools/calib_traffic.hip -o tools/bin/calib_traffic
// run:   rocprofv3 --pmc FETCH_SIZE -- tools/bin/calib_traffic ; rocprofv3 --pmc WRITE_SIZE -- tools/bin/calib_traffic
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                             \
    do {                                                                                                  \
        hipError_t e_ = (x);                                                                              \
        if (e_ != hipSuccess) {                                                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                       \
            exit(1);                                                                                      \
        }                                                                                                 \
    } while (0)

static constexpr size_t kBytes = size_t(2) << 30;   // 2 GiB per buffer

__global__ void read16(const float4* __restrict__ a, size_t n, float* __restrict__ sink) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) sink[0] = s;   // never true for the zero-filled input: keeps the loads
}
__global__ void read8(const float2* __restrict__ a, size_t n, float* __restrict__ sink) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 12345.f) sink[0] = s;
}
__global__ void read4(const int* __restrict__ a, size_t n, float* __restrict__ sink) {
    int s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 12345) sink[0] = (float)s;
}
__global__ void write16(float4* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}
__global__ void write4(int* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = (int)i;
}
// one 4-B store into each 128-B line (32 ints apart)
__global__ void scat4(int* __restrict__ a, size_t lines) {
    for (size_t l = blockIdx.x * (size_t)blockDim.x + threadIdx.x; l < lines; l += (size_t)gridDim.x * blockDim.x)
        a[l * 32 + (l % 32)] = (int)l;
}
// column-major [64][N] int list; one wave per row r (every `step`-th row), lane t stores column t
__global__ void rowcol4(int* __restrict__ a, size_t N, size_t step) {
    const int lane = threadIdx.x & 63;
    const size_t w0 = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t r = w0 * step; r < N; r += nw * step) a[(size_t)lane * N + r] = (int)r;
}
// random 16-B row gathers (hash of the thread index), each row of the table at most ~once
__global__ void gath16(const float4* __restrict__ t, size_t rows, size_t n, float* __restrict__ sink) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = (i * 2654435761ull) % rows;   // a permutation of [0, rows) for rows coprime to the multiplier
        const float4 v = t[r];
        s += v.x;
    }
    if (s == 12345.f) sink[0] = s;
}

int main() {
    char *a = nullptr, *b = nullptr;
    float* sink = nullptr;
    CK(hipMalloc(&a, kBytes));
    CK(hipMalloc(&b, kBytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 0, kBytes));
    CK(hipMemset(b, 0, kBytes));
    CK(hipDeviceSynchronize());
    const dim3 blk(256), grd(8192);
    // a second pass over b between tests evicts a from the Infinity Cache (256 MiB)
    auto flush = [&]() { hipLaunchKernelGGL(write4, grd, blk, 0, 0, (int*)b, kBytes / 4); };
    hipLaunchKernelGGL(read16, grd, blk, 0, 0, (const float4*)a, kBytes / 16, sink);   flush();
    hipLaunchKernelGGL(read8, grd, blk, 0, 0, (const float2*)a, kBytes / 8, sink);     flush();
    hipLaunchKernelGGL(read4, grd, blk, 0, 0, (const int*)a, kBytes / 4, sink);        flush();
    hipLaunchKernelGGL(write16, grd, blk, 0, 0, (float4*)a, kBytes / 16);              flush();
    hipLaunchKernelGGL(write4, grd, blk, 0, 0, (int*)a, kBytes / 4);                   flush();
    hipLaunchKernelGGL(scat4, grd, blk, 0, 0, (int*)a, kBytes / 128);                  flush();
    const size_t N = kBytes / 4 / 64;   // rows of a [64][N] int list filling the buffer
    hipLaunchKernelGGL(rowcol4, grd, blk, 0, 0, (int*)a, N, (size_t)16);               flush();
    const size_t rows = kBytes / 16 - 1;   // odd: coprime to the (odd) multiplier's factors in practice
    hipLaunchKernelGGL(gath16, grd, blk, 0, 0, (const float4*)a, rows, rows / 8, sink);
    CK(hipDeviceSynchronize());
    printf("true bytes: read16 %zu read8 %zu read4 %zu write16 %zu write4 %zu scat4 %zu (4 B per 128-B line) "
           "rowcol4 %zu (64 x 4 B per 16th row) gath16 %zu (16 B rows)\n",
           kBytes, kBytes, kBytes, kBytes, kBytes, (kBytes / 128) * 4, (N / 16) * 64 * 4, (rows / 8) * 16);
    printf("flush = write4 over another 2 GiB buffer (true bytes %zu)\n", kBytes);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(sink));
    return 0;
}
