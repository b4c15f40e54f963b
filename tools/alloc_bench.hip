// How long does mapping a whole-HBM arena take?  hipMalloc vs the virtual
// memory API (one physical handle, or 1 GiB handles) vs a stream-ordered pool.
// Each allocation is followed by a memset so lazily mapped pages are counted.
// build: hipcc -O2 --offload-arch=gfx950 tools/alloc_bench.hip -o tools/alloc_bench
// run:   tools/alloc_bench [GB]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));                \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

static double now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

static void touch(void *p, size_t bytes, const char *what, double t_alloc) {
    double t0 = now_ms();
    CK(hipMemsetAsync(p, 0, bytes, nullptr));
    CK(hipStreamSynchronize(nullptr));
    std::printf("{\"api\": \"%s\", \"GB\": %.1f, \"alloc_ms\": %.1f, \"memset_ms\": %.1f}\n", what, bytes / 1e9,
                t_alloc, now_ms() - t0);
    std::fflush(stdout);
}

int main(int argc, char **argv) {
    const double gb = argc > 1 ? std::atof(argv[1]) : 240.0;
    const size_t gib = size_t(1) << 30;
    size_t bytes = size_t(gb * 1e9) / gib * gib;
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));

    for (int rep = 0; rep < 2; ++rep) {
        void *p = nullptr;
        double t0 = now_ms();
        CK(hipMalloc(&p, bytes));
        double ta = now_ms() - t0;
        touch(p, bytes, "hipMalloc", ta);
        t0 = now_ms();
        CK(hipFree(p));
        std::printf("{\"api\": \"hipFree\", \"ms\": %.1f}\n", now_ms() - t0);
    }

    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    std::printf("{\"granularity\": %zu}\n", gran);
    for (size_t chunk : {bytes, gib * 4, gib}) {
        double t0 = now_ms();
        hipDeviceptr_t base = nullptr;
        CK(hipMemAddressReserve((void **)&base, bytes, 0, nullptr, 0));
        std::vector<hipMemGenericAllocationHandle_t> hs;
        for (size_t off = 0; off < bytes; off += chunk) {
            size_t n = std::min(chunk, bytes - off);
            hipMemGenericAllocationHandle_t h;
            CK(hipMemCreate(&h, n, &prop, 0));
            CK(hipMemMap((char *)base + off, n, 0, h, 0));
            hs.push_back(h);
        }
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        CK(hipMemSetAccess(base, bytes, &acc, 1));
        double ta = now_ms() - t0;
        char name[64];
        std::snprintf(name, sizeof name, "vmm chunk %zu GiB", chunk / gib);
        touch(base, bytes, name, ta);
        t0 = now_ms();
        CK(hipMemUnmap(base, bytes));
        for (auto h : hs) CK(hipMemRelease(h));
        CK(hipMemAddressFree(base, bytes));
        std::printf("{\"api\": \"vmm free\", \"ms\": %.1f}\n", now_ms() - t0);
    }

    {
        hipMemPool_t pool;
        CK(hipDeviceGetDefaultMemPool(&pool, 0));
        uint64_t thr = UINT64_MAX;
        CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
        for (int rep = 0; rep < 2; ++rep) {
            void *p = nullptr;
            double t0 = now_ms();
            CK(hipMallocAsync(&p, bytes, nullptr));
            CK(hipStreamSynchronize(nullptr));
            double ta = now_ms() - t0;
            touch(p, bytes, rep ? "hipMallocAsync (pool warm)" : "hipMallocAsync", ta);
            CK(hipFreeAsync(p, nullptr));
            CK(hipStreamSynchronize(nullptr));
        }
    }
    return 0;
}
