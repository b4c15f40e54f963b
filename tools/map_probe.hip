// Where does a cold 32x32 MAR's arena mapping go?  Per-chunk timings of
// mapping ~240 GB of HBM in 8-GiB pieces: (a) first thing in a fresh process,
// (b) right after this process freed it, (c) after 5 s and (d) 20 s of quiet,
// (e) the same through the virtual-memory API (hipMemCreate + hipMemMap), and
// (f) what a second thread's kernel launches, small hipMalloc and small
// hipMemcpy cost while a helper thread maps dirty chunks.
// build: hipcc -O2 --offload-arch=gfx950 tools/map_probe.hip -o tools/map_probe -lpthread
// run:   tools/map_probe [GB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <unistd.h>
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

__global__ void spin_kernel(float *p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 1.0001f + 1.0f;
}

static const size_t kChunk = size_t(8) << 30;

static std::vector<void *> map_chunks(int n, const char *tag) {
    std::vector<void *> ps;
    std::printf("{\"phase\": \"%s\", \"chunk_GiB\": 8, \"ms\": [", tag);
    double tot = 0;
    for (int i = 0; i < n; ++i) {
        void *p = nullptr;
        double t0 = now_ms();
        CK(hipMalloc(&p, kChunk));
        double dt = now_ms() - t0;
        tot += dt;
        std::printf("%s%.1f", i ? ", " : "", dt);
        ps.push_back(p);
    }
    std::printf("], \"total_ms\": %.1f, \"GB_per_s\": %.1f}\n", tot, n * (double)kChunk / 1e9 / (tot / 1e3));
    std::fflush(stdout);
    return ps;
}

static void touch_all(std::vector<void *> &ps, const char *tag) {
    double t0 = now_ms();
    for (void *p : ps) CK(hipMemsetAsync(p, 0, kChunk, nullptr));
    CK(hipStreamSynchronize(nullptr));
    std::printf("{\"phase\": \"%s memset\", \"ms\": %.1f}\n", tag, now_ms() - t0);
    std::fflush(stdout);
}

static void free_all(std::vector<void *> &ps) {
    double t0 = now_ms();
    for (void *p : ps) CK(hipFree(p));
    ps.clear();
    std::printf("{\"phase\": \"free\", \"ms\": %.1f}\n", now_ms() - t0);
    std::fflush(stdout);
}

int main(int argc, char **argv) {
    const double gb = argc > 1 ? std::atof(argv[1]) : 240.0;
    const int n = std::max(1, (int)(gb * 1e9 / kChunk));
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    size_t fr = 0, tot = 0;
    CK(hipMemGetInfo(&fr, &tot));
    std::printf("{\"free_GB\": %.1f, \"total_GB\": %.1f, \"chunks\": %d}\n", fr / 1e9, tot / 1e9, n);

    auto ps = map_chunks(n, "a fresh process");
    touch_all(ps, "a");
    free_all(ps);
    ps = map_chunks(n, "b right after free");
    free_all(ps);
    sleep(5);
    ps = map_chunks(n, "c after 5 s");
    free_all(ps);
    sleep(20);
    ps = map_chunks(n, "d after 20 s more");
    touch_all(ps, "d");
    free_all(ps);

    // (e) virtual-memory API, dirty again
    {
        hipMemAllocationProp prop = {};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = 0;
        const size_t bytes = (size_t)n * kChunk;
        hipDeviceptr_t base = nullptr;
        double t0 = now_ms();
        CK(hipMemAddressReserve((void **)&base, bytes, 0, nullptr, 0));
        double tr = now_ms() - t0;
        std::vector<hipMemGenericAllocationHandle_t> hs;
        std::printf("{\"phase\": \"e vmm\", \"reserve_ms\": %.2f, \"create_map_access_ms\": [", tr);
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        for (int i = 0; i < n; ++i) {
            hipMemGenericAllocationHandle_t h;
            double a = now_ms();
            CK(hipMemCreate(&h, kChunk, &prop, 0));
            double b = now_ms();
            CK(hipMemMap((char *)base + (size_t)i * kChunk, kChunk, 0, h, 0));
            double c = now_ms();
            CK(hipMemSetAccess((char *)base + (size_t)i * kChunk, kChunk, &acc, 1));
            double d = now_ms();
            std::printf("%s[%.1f, %.1f, %.1f]", i ? ", " : "", b - a, c - b, d - c);
            hs.push_back(h);
        }
        std::printf("]}\n");
        std::fflush(stdout);
        t0 = now_ms();
        CK(hipMemsetAsync((void *)base, 0, bytes, nullptr));
        CK(hipStreamSynchronize(nullptr));
        std::printf("{\"phase\": \"e memset\", \"ms\": %.1f}\n", now_ms() - t0);
        t0 = now_ms();
        CK(hipMemUnmap(base, bytes));
        for (auto h : hs) CK(hipMemRelease(h));
        CK(hipMemAddressFree(base, bytes));
        std::printf("{\"phase\": \"e vmm free\", \"ms\": %.1f}\n", now_ms() - t0);
        std::fflush(stdout);
    }

    // (f) a helper thread maps (dirty) chunks; the main thread launches small
    // kernels, small hipMallocs and small copies meanwhile
    {
        float *work = nullptr;
        const int nw = 1 << 20;
        CK(hipMalloc(&work, nw * sizeof(float)));
        hipStream_t st;
        CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        std::vector<char> host(1 << 20, 1);
        std::atomic<int> done{0};
        std::vector<void *> hp;
        double t_start = now_ms();
        std::thread helper([&]() {
            CK(hipSetDevice(0));
            for (int i = 0; i < n; ++i) {
                void *p = nullptr;
                CK(hipMalloc(&p, kChunk));
                hp.push_back(p);
            }
            done = 1;
        });
        double max_launch = 0, max_small_alloc = 0, max_copy = 0, sum_launch = 0;
        int launches = 0, allocs = 0;
        while (!done) {
            double a = now_ms();
            hipLaunchKernelGGL(spin_kernel, dim3(nw / 256), dim3(256), 0, st, work, nw);
            double b = now_ms();
            max_launch = std::max(max_launch, b - a);
            sum_launch += b - a;
            ++launches;
            if (launches % 50 == 0) {
                void *q = nullptr;
                double c = now_ms();
                CK(hipMalloc(&q, 1 << 20));
                double d = now_ms();
                CK(hipMemcpy(q, host.data(), host.size(), hipMemcpyHostToDevice));
                double e = now_ms();
                CK(hipFree(q));
                max_small_alloc = std::max(max_small_alloc, d - c);
                max_copy = std::max(max_copy, e - d);
                ++allocs;
            }
            if (launches % 200 == 0) CK(hipStreamSynchronize(st));
        }
        helper.join();
        CK(hipStreamSynchronize(st));
        std::printf("{\"phase\": \"f concurrent\", \"helper_map_ms\": %.1f, \"launches\": %d, \"mean_launch_ms\": %.3f, "
                    "\"max_launch_ms\": %.1f, \"small_allocs\": %d, \"max_small_alloc_ms\": %.1f, \"max_small_copy_ms\": %.1f}\n",
                    now_ms() - t_start, launches, sum_launch / std::max(1, launches), max_launch, allocs, max_small_alloc,
                    max_copy);
        std::fflush(stdout);
        free_all(hp);
        CK(hipFree(work));
    }
    return 0;
}
