// Host-side plumbing shared by the libpcd translation units: status/error handling, the grid object, and the
// device view of the grid that kernels receive by value.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/pcd.h"

namespace pcd {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define PCD_CHECK_ARG(cond, msg) \
    do { if (!(cond)) return ::pcd::fail(PCD_ERR_ARG, std::string(__func__) + ": " + (msg)); } while (0)
#define PCD_HIP(call)                                                                                      \
    do {                                                                                                   \
        hipError_t e_ = (call);                                                                            \
        if (e_ != hipSuccess) {                                                                            \
            return ::pcd::fail(e_ == hipErrorOutOfMemory ? PCD_ERR_OOM : PCD_ERR_HIP,                      \
                               std::string(__func__) + ": " #call ": " + hipGetErrorString(e_));          \
        }                                                                                                  \
    } while (0)
#define PCD_LAUNCH_CHECK() PCD_HIP(hipGetLastError())

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Stream-ordered temporaries of one entry point: every pointer taken through alloc() is released with hipFreeAsync
// on every exit path (an early PCD_HIP / PCD_CHECK_ARG return included), and the destructor then synchronises the
// stream so no caller sees a call return with its scratch still in use.
struct StreamTemps {
    hipStream_t st;
    void* p[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    int n = 0;
    explicit StreamTemps(hipStream_t s) : st(s) {}
    template <class T>
    hipError_t alloc(T** out, size_t bytes) {
        *out = nullptr;
        if (n == 8) return hipErrorInvalidValue;
        void* q = nullptr;
        const hipError_t e = hipMallocAsync(&q, bytes, st);
        if (e == hipSuccess) { p[n++] = q; *out = static_cast<T*>(q); }
        return e;
    }
    // free everything now (stream-ordered; sync: and wait for the stream), reporting the first failure
    hipError_t release(bool sync = true) {
        hipError_t first = hipSuccess;
        for (int i = 0; i < n; ++i) {
            const hipError_t e = hipFreeAsync(p[i], st);
            if (first == hipSuccess) first = e;
            p[i] = nullptr;
        }
        n = 0;
        const hipError_t e = sync ? hipStreamSynchronize(st) : hipSuccess;
        return first == hipSuccess ? e : first;
    }
    ~StreamTemps() { if (n) (void)release(); }
    StreamTemps(const StreamTemps&) = delete;
    StreamTemps& operator=(const StreamTemps&) = delete;
};
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// One 16-byte hash slot: Morton key of an occupied cell -> [start, end) in the sorted snapshot.
struct HashSlot {            // one occupied BRICK (4x4x4 cells): Morton brick key -> brick index
    unsigned long long key;
    uint32_t brick, pad;
};
static constexpr unsigned long long kEmptyKey = ~0ull;

// Kernel-side view of a grid (passed by value).
struct GridView {
    const float4* pts;       // snapshot, Morton-sorted, w unused
    const HashSlot* table;   // occupied bricks (open addressing, load <= 1/2)
    const uint2* cells;      // [bricks][64] (start, end) snapshot rows of each cell; start == end: empty
    unsigned long long mask; // table slots - 1
    int hbits;               // log2(slots)
    float ox, oy, oz, h, inv_h;
    int dx, dy, dz;
    int64_t n;
    float slack;             // bound on how far a row can sit outside its cell box (fp32 rounding of the keys)
};

}  // namespace pcd

struct pcd_grid {
    int device = 0;
    int64_t n = 0;
    int64_t cells = 0;
    float4* pts = nullptr;     // [n]
    int32_t* perm = nullptr;   // [n] sorted rank -> original index
    pcd::HashSlot* table = nullptr;
    uint2* cellr = nullptr;    // [bricks][64]
    int64_t slots = 0;
    int64_t bricks = 0;
    pcd::GridView view{};
};
