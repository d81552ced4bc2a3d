// vbf_api.hip -- the C ABI (include/vbf.h) over the gfx950 kernels.
//
// Host-side responsibilities: argument checks that mirror the reference's asserts/panics,
// sizing arithmetic (bf.rs:230-239), the filter handle (bf.rs:38-58 semantics: clones share
// one bit array behind a mutex, like Arc<Mutex<BitVec>>), and the chunked, double-buffered
// H2D pipeline for keys that arrive in host memory (memtable / compaction output).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <utility>
#include <atomic>
#include <cstdarg>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "../../include/vbf.h"
#include "sip13.hpp"
#include "vbf_kernels.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

inline int ok() {
    g_err.clear();
    return VBF_OK;
}

// On failure the thread's sticky HIP error is cleared (hipGetLastError resets it) after it is
// reported, so it cannot resurface as a later launch's hipGetLastError on the same thread -- e.g.
// the next asynchronous set a device's worker thread runs after one whose allocation failed.
#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) {                                                               \
            (void)hipGetLastError();                                                          \
            int code_ = (e_ == hipErrorOutOfMemory) ? VBF_ENOMEM : VBF_EHIP;                  \
            return fail(code_, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
        }                                                                                     \
    } while (0)

// Switches the calling thread to `device` for the scope, restoring the previous one.
// HIP does not survive fork(): a child of a process that used the GPU through this library must not
// call into HIP (such calls can hang or fault).  The first device scope records the process that
// uses HIP; a forked child's device scopes fail with VBF_EINVAL before any HIP call.
std::atomic<pid_t> g_hip_pid{0};

bool hip_forked() {
    const pid_t owner = g_hip_pid.load();
    return owner != 0 && owner != getpid();
}

// Records the calling process as the one that uses HIP (the first call wins); false in a child
// forked from it.
bool hip_owner() {
    const pid_t me = getpid();
    pid_t owner = 0;
    return g_hip_pid.compare_exchange_strong(owner, me) || owner == me;
}

int fail_forked() {
    return fail(VBF_EINVAL, "process %d forked from %d, which uses the GPU: HIP cannot be used in the child",
                (int)getpid(), (int)g_hip_pid.load());
}

// The stateless device-pointer entry points (no DeviceGuard: they run on the caller's current
// device) check the same at their start.
#define FORK_GUARD()                          \
    do {                                      \
        if (!hip_owner()) return fail_forked(); \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    bool forked = false;
    explicit DeviceGuard(int device) {
        if (!hip_owner()) {
            forked = true;
            err = hipErrorNotSupported;
            return;
        }
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != device) err = hipSetDevice(device);
    }
    ~DeviceGuard() {
        if (forked) return;
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

#define DEVICE_SCOPE(dev)                                                                     \
    DeviceGuard guard_(dev);                                                                  \
    if (guard_.forked) return fail_forked();                                                  \
    if (guard_.err != hipSuccess)                                                             \
        return fail(VBF_ENODEV, "hipSetDevice(%d): %s", (int)(dev), hipGetErrorString(guard_.err))

// Rust `f64 as u32`: saturating, NaN -> 0, truncation toward zero.
uint32_t f64_as_u32(double x) {
    if (std::isnan(x) || x <= 0.0) return 0;
    if (x >= 4294967295.0) return 4294967295u;
    return (uint32_t)x;
}

int check_keys(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n) {
    if (n == 0) return VBF_OK;
    if (!keys && !offsets && stride) return fail(VBF_EINVAL, "keys is NULL");
    if (offsets == nullptr && stride == 0) return VBF_OK;  // n empty keys
    return VBF_OK;
}

int check_mk(uint32_t m, uint32_t k, uint64_t n) {
    if (m == 0 && k > 0 && n > 0)
        return fail(VBF_EDIVZERO, "m == 0 with k = %u > 0: the reference divides by zero (bf.rs:88)", k);
    return VBF_OK;
}

vbf::KeyBatch batch(const uint8_t* keys, const uint64_t* offsets, uint64_t off_base,
                    uint64_t stride, uint64_t n, int lp) {
    return vbf::KeyBatch{keys, offsets, off_base, stride, n, lp != 0};
}

// ---------------------------------------------------------------------------------------
// Partitioned-build workspace: one grow-only buffer per (device, stream), so concurrent
// builds on different streams never share scratch.
// ---------------------------------------------------------------------------------------
enum WsSlot {
    kWsBuild = 0,
    kWsSstScratch = 1,
    kWsSstKeys = 2,
    kWsSstInput = 3,
    kWsMulti = 4,
    kWsMultiKeys = 5,
    kWsCompact = 6,
    kWsCompactIn = 7,
    kWsGather = 8,
    kWsProbe = 9,
    kWsCount = 10,
    kWsMultiGroup = 11,
};
struct Workspace {
    int device;
    hipStream_t stream;
    int slot;
    void* ptr;
    uint64_t bytes;
};
std::mutex g_ws_mu;
std::vector<Workspace> g_ws;

// VBF_WS_MAX_BYTES (read per call): the largest single workspace the library may allocate -- for a
// caller sharing the GPU; a build whose default chunk needs more runs in smaller chunks (do_build)
uint64_t ws_max_bytes() {
    const char* e = getenv("VBF_WS_MAX_BYTES");
    return e ? strtoull(e, nullptr, 10) : ~0ull;
}

int get_workspace(hipStream_t s, uint64_t bytes, void** out, int slot = kWsBuild) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    bytes = std::max<uint64_t>(bytes, 256);
    if (bytes > ws_max_bytes())
        return fail(VBF_ENOMEM, "workspace of %llu bytes above VBF_WS_MAX_BYTES", (unsigned long long)bytes);
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (auto& w : g_ws) {
        if (w.device == dev && w.stream == s && w.slot == slot) {
            if (w.bytes < bytes) {
                HIP_TRY(hipStreamSynchronize(s));  // the old buffer may still be in use on s
                HIP_TRY(hipFree(w.ptr));
                w.ptr = nullptr;
                w.bytes = 0;
                HIP_TRY(hipMalloc(&w.ptr, bytes));
                w.bytes = bytes;
            }
            *out = w.ptr;
            return VBF_OK;
        }
    }
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, bytes));
    g_ws.push_back(Workspace{dev, s, slot, p, bytes});
    *out = p;
    return VBF_OK;
}

constexpr uint64_t kAutoPartitionMinIdx = 1ull << 22;
// batched multi-SST probe: below this many keys every filter is probed one lane per key
constexpr uint64_t kMultiGroupMinKeys = 1ull << 20;

// The build every entry point funnels into.  strategy: VBF_BUILD_AUTO / _ATOMIC / _PARTITIONED.
// atomic_merge: another writer may touch `words` concurrently (the partitioned path then
// merges its segments with word atomics instead of load+store).
int do_build(const vbf::KeyBatch& kb, uint32_t m, uint32_t k, uint32_t* words, int strategy,
             bool atomic_merge, hipStream_t s) {
    const bool fresh = (strategy & VBF_BUILD_FRESH) != 0;
    strategy &= ~VBF_BUILD_FRESH;
    // a fresh filter the segment pass cannot write whole (atomic strategy, no keys, several
    // chunks or several workgroups per segment) is zeroed first: BitVec::from_elem(m, false)
    auto zero = [&]() -> int {
        if (fresh && m) HIP_TRY(hipMemsetAsync(words, 0, ((uint64_t)m + 31) / 32 * 4, s));
        return VBF_OK;
    };
    if (kb.n == 0 || k == 0) return zero();
    bool part;
    if (strategy == VBF_BUILD_ATOMIC) {
        part = false;
    } else if (strategy == VBF_BUILD_PARTITIONED) {
        if (!vbf::partition_supported(m, k))
            return fail(VBF_EINVAL, "partitioned build needs 1 <= k <= 32 and m > 0 (k = %u)", k);
        part = true;
    } else if (strategy == VBF_BUILD_AUTO) {
        part = vbf::partition_supported(m, k) && kb.n * (uint64_t)k >= kAutoPartitionMinIdx;
    } else {
        return fail(VBF_EINVAL, "unknown build strategy %d", strategy);
    }
    if (!part) {
        if (int rc = zero()) return rc;
        HIP_TRY(vbf::launch_build(kb, m, k, words, s));
        return VBF_OK;
    }
    // The workspace holds one chunk of bit indices (kBuildChunkIdx = 2^32: ~10.7 GB).  When it
    // cannot be allocated (other streams' workspaces, the caller's own memory), the chunk is halved
    // down to 2^28 indices -- more segment passes, the same words.
    uint64_t chunk = vbf::build_chunk_default(), need = 0;
    void* ws = nullptr;
    for (;;) {
        need = vbf::partition_workspace_bytes(kb.n, m, k, chunk);
        const int rc = get_workspace(s, need, &ws);
        if (rc == VBF_OK) break;
        if (rc != VBF_ENOMEM || chunk <= (1ull << 28)) return rc;
        chunk /= 2;
    }
    const bool fused = fresh && !atomic_merge && vbf::partition_fresh_ok(kb.n, m, k, chunk);
    if (fresh && !fused)
        if (int rc = zero()) return rc;
    HIP_TRY(vbf::launch_build_partitioned(kb, m, k, words, ws, need, atomic_merge, s, fused, chunk));
    return VBF_OK;
}

// The probe every entry point funnels into: out (answer bytes) or count (hits).  The per-key
// early-exit gather costs ~1 + (k-1)*hit_rate random filter loads per key; the partitioned probe
// costs all k hashes per key but no random loads.  AUTO (large batches over large filters) probes
// the first 64K keys with the gather, reads the hit count back (one stream sync) and takes the
// partitioned path when at least 35 % of them hit (measured crossover: 100M keys, k = 10).
constexpr uint64_t kAutoProbePartitionMinIdx = 1ull << 24;
constexpr uint64_t kProbeSample = 1ull << 16;

int do_probe(const vbf::KeyBatch& kb, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
             unsigned long long* count, int strategy, hipStream_t s) {
    if (kb.n == 0) return VBF_OK;
    bool part;
    if (strategy == VBF_BUILD_ATOMIC) {
        part = false;
    } else if (strategy == VBF_BUILD_PARTITIONED) {
        if (!vbf::probe_partition_supported(m, k))
            return fail(VBF_EINVAL, "partitioned probe needs 1 <= k <= 32 and a filter of at least 1 segment (k = %u)", k);
        part = true;
    } else if (strategy == VBF_BUILD_AUTO) {
        part = k > 1 && vbf::probe_partition_supported(m, k) && kb.n * (uint64_t)k >= kAutoProbePartitionMinIdx &&
               m >= (64u << 20);
        if (part) {  // sample the hit rate
            vbf::KeyBatch sb = kb;
            sb.n = std::min<uint64_t>(kb.n, kProbeSample);
            const uint64_t np = vbf::count_partials(sb.n);
            void* pw = nullptr;
            int rc = get_workspace(s, np * 4 + 256, &pw, kWsCount);
            if (rc) return rc;
            auto* c = reinterpret_cast<unsigned long long*>(static_cast<char*>(pw) + np * 4);
            c = reinterpret_cast<unsigned long long*>(((uintptr_t)c + 7) & ~(uintptr_t)7);
            HIP_TRY(hipMemsetAsync(c, 0, 8, s));
            HIP_TRY(vbf::launch_count(sb, m, k, words, c, static_cast<uint32_t*>(pw), s));
            unsigned long long hits = 0;
            HIP_TRY(hipMemcpyAsync(&hits, c, 8, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            part = hits * 100 >= sb.n * 35;
        }
    } else {
        return fail(VBF_EINVAL, "unknown probe strategy %d", strategy);
    }
    if (!part || k == 0) {
        if (count) {
            void* pw = nullptr;
            int rc = get_workspace(s, vbf::count_partials(kb.n) * 4, &pw, kWsCount);
            if (rc) return rc;
            HIP_TRY(vbf::launch_count(kb, m, k, words, count, static_cast<uint32_t*>(pw), s));
        } else {
            HIP_TRY(vbf::launch_probe(kb, m, k, words, out, s));
        }
        return VBF_OK;
    }
    const uint64_t need = vbf::probe_workspace_bytes(kb.n, m, k);
    void* ws = nullptr;
    int rc = get_workspace(s, need, &ws, kWsProbe);
    if (rc) return rc;
    HIP_TRY(vbf::launch_probe_partitioned(kb, m, k, words, out, count, ws, need, s));
    return VBF_OK;
}

// ---------------------------------------------------------------------------------------
// Host -> device staging: two pinned buffers and two streams per device; chunk c uses
// buffer (c & 1), so the H2D copy of chunk c+1 overlaps the kernel of chunk c.
// ---------------------------------------------------------------------------------------
constexpr uint64_t kChunkBytes = 64ull << 20;

// Host copy into / out of the pinned staging buffers, split over up to 8 threads
// (VBF_COPY_THREADS): one thread's memcpy into pinned memory runs well below the PCIe rate.  The
// helper threads are a persistent pool (creating 7 threads per 16 MiB chunk cost ~0.1 ms each
// chunk); concurrent callers take turns.
class CopyPool {
  public:
    static CopyPool& get() {
        static std::mutex mu;
        static CopyPool* p = nullptr;  // never destroyed: workers outlive static teardown
        std::lock_guard<std::mutex> lk(mu);
        // a forked child (e.g. a multiprocessing fork) inherits the pool but not its threads:
        // it gets a pool of its own
        if (!p || p->pid_ != getpid()) p = new CopyPool();
        return *p;
    }
    unsigned threads() const { return nt_; }
    // Runs f(0 .. parts-1) with part 0 on the calling thread.
    template <class F>
    void run(unsigned parts, F&& f) {
        std::lock_guard<std::mutex> caller(call_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = [&f](unsigned i) { f(i); };
            parts_ = parts;
            next_ = 1;
            done_ = 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return done_ == parts_; });
        job_ = nullptr;
    }

  private:
    CopyPool() : pid_(getpid()) {
        const char* e = getenv("VBF_COPY_THREADS");
        const unsigned hw = std::thread::hardware_concurrency();
        const int v = e ? atoi(e) : (int)std::min(8u, hw ? hw : 1u);
        nt_ = (unsigned)std::max(1, v);
        for (unsigned t = 1; t < nt_; ++t) std::thread([this] { loop(); }).detach();
    }
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return gen_ != seen; });
            seen = gen_;
            while (next_ < parts_) {
                const unsigned i = next_++;
                auto job = job_;
                lk.unlock();
                job(i);
                lk.lock();
                if (++done_ == parts_) done_cv_.notify_one();
            }
        }
    }
    const pid_t pid_;
    unsigned nt_ = 1;
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    std::function<void(unsigned)> job_;
    unsigned parts_ = 0, next_ = 0, done_ = 0;
    uint64_t gen_ = 0;
};

void par_memcpy(void* dst, const void* src, size_t n) {
    constexpr size_t kMinPerThread = 2u << 20;
    CopyPool& pool = CopyPool::get();
    const unsigned nt = (unsigned)std::min<size_t>(pool.threads(), n / kMinPerThread);
    if (nt <= 1) {
        std::memcpy(dst, src, n);
        return;
    }
    const size_t per = (n / nt + 4095) & ~(size_t)4095;
    pool.run(nt, [=](unsigned t) {
        const size_t a = (size_t)t * per;
        if (a < n) std::memcpy(static_cast<char*>(dst) + a, static_cast<const char*>(src) + a, std::min(per, n - a));
    });
}

struct Staging {
    std::mutex mu;
    int device = -1;
    hipStream_t stream[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    uint8_t* h_keys[2] = {nullptr, nullptr};
    uint8_t* d_keys[2] = {nullptr, nullptr};
    uint64_t key_cap[2] = {0, 0};
    uint64_t* h_offs[2] = {nullptr, nullptr};
    uint64_t* d_offs[2] = {nullptr, nullptr};
    uint64_t off_cap[2] = {0, 0};
    uint8_t* h_out[2] = {nullptr, nullptr};
    uint8_t* d_out[2] = {nullptr, nullptr};
    uint64_t out_cap[2] = {0, 0};
    uint32_t* d_words = nullptr;  // scratch filter for the one-shot host API
    uint64_t words_cap = 0;
    uint8_t* h_xfer[2] = {nullptr, nullptr};  // pinned bounce buffers for large filter copies
    hipEvent_t first = nullptr;  // a fresh filter's first chunk built: the other chunks OR after it

    int init(int dev) {
        if (device == dev) return VBF_OK;
        device = dev;
        for (int b = 0; b < 2; ++b) {
            HIP_TRY(hipStreamCreateWithFlags(&stream[b], hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&done[b], hipEventDisableTiming));
        }
        HIP_TRY(hipEventCreateWithFlags(&first, hipEventDisableTiming));
        return VBF_OK;
    }
    template <class T>
    static int grow(T** h, T** d, uint64_t* cap, uint64_t count) {
        if (count <= *cap) return VBF_OK;
        if (h && *h) HIP_TRY(hipHostFree(*h));
        if (*d) HIP_TRY(hipFree(*d));
        if (h) *h = nullptr;
        *d = nullptr;
        *cap = 0;
        uint64_t want = count + count / 4 + 64;
        if (h) HIP_TRY(hipHostMalloc((void**)h, want * sizeof(T), hipHostMallocDefault));
        HIP_TRY(hipMalloc((void**)d, want * sizeof(T)));
        *cap = want;
        return VBF_OK;
    }
};

// Large host <-> device copies (filter words) bounce through two pinned chunk buffers, so the
// DMA of chunk c+1 overlaps the (threaded) host copy of chunk c; pageable hipMemcpy runs at a
// fraction of the link rate.  Small copies go direct.  Caller holds st.mu and has ordered src.
constexpr uint64_t kXferDirect = 8ull << 20;
// bounce chunk: small enough that the last chunk's host copy (not overlapped) is short
constexpr uint64_t kXferChunk = 16ull << 20;

int xfer_bufs(Staging& st) {
    for (int b = 0; b < 2; ++b)
        if (!st.h_xfer[b]) HIP_TRY(hipHostMalloc((void**)&st.h_xfer[b], kChunkBytes, hipHostMallocDefault));
    return VBF_OK;
}

bool d2h_direct() {  // VBF_D2H_DIRECT=1: pageable hipMemcpy instead of the bounce (A/B)
    static const bool v = [] { const char* e = getenv("VBF_D2H_DIRECT"); return e && atoi(e) != 0; }();
    return v;
}

int xfer_d2h(Staging& st, void* dst, const void* src, uint64_t bytes) {
    if (bytes < kXferDirect || d2h_direct()) {
        HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
        return VBF_OK;
    }
    int rc = xfer_bufs(st);
    if (rc) return rc;
    const uint64_t nc = (bytes + kXferChunk - 1) / kXferChunk;
    for (uint64_t c = 0; c <= nc; ++c) {
        if (c < nc) {
            const int b = (int)(c & 1);
            const uint64_t off = c * kXferChunk, len = std::min<uint64_t>(kXferChunk, bytes - off);
            HIP_TRY(hipMemcpyAsync(st.h_xfer[b], static_cast<const char*>(src) + off, len, hipMemcpyDeviceToHost,
                                   st.stream[b]));
            HIP_TRY(hipEventRecord(st.done[b], st.stream[b]));
        }
        if (c > 0) {
            const int pb = (int)((c - 1) & 1);
            const uint64_t off = (c - 1) * kXferChunk, len = std::min<uint64_t>(kXferChunk, bytes - off);
            HIP_TRY(hipEventSynchronize(st.done[pb]));
            par_memcpy(static_cast<char*>(dst) + off, st.h_xfer[pb], len);
        }
    }
    return VBF_OK;
}

// H2D on st.stream[0..1]; returns with both streams synchronized.
int xfer_h2d(Staging& st, void* dst, const void* src, uint64_t bytes) {
    if (bytes < kXferDirect) {
        HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
        return VBF_OK;
    }
    int rc = xfer_bufs(st);
    if (rc) return rc;
    const uint64_t nc = (bytes + kXferChunk - 1) / kXferChunk;
    for (uint64_t c = 0; c < nc; ++c) {
        const int b = (int)(c & 1);
        const uint64_t off = c * kXferChunk, len = std::min<uint64_t>(kXferChunk, bytes - off);
        if (c >= 2) HIP_TRY(hipEventSynchronize(st.done[b]));  // buffer b's previous DMA finished
        par_memcpy(st.h_xfer[b], static_cast<const char*>(src) + off, len);
        HIP_TRY(hipMemcpyAsync(static_cast<char*>(dst) + off, st.h_xfer[b], len, hipMemcpyHostToDevice, st.stream[b]));
        HIP_TRY(hipEventRecord(st.done[b], st.stream[b]));
    }
    for (int b = 0; b < 2; ++b) HIP_TRY(hipStreamSynchronize(st.stream[b]));
    return VBF_OK;
}

// VBF_H2D_DIRECT=0 forces the pinned bounce for key chunks (A/B); default: direct.
bool h2d_direct() {
    static const bool v = [] { const char* e = getenv("VBF_H2D_DIRECT"); return !e || atoi(e) != 0; }();
    return v;
}

std::mutex g_staging_mu;
std::vector<std::unique_ptr<Staging>> g_staging;

Staging* staging_for(int device) {
    std::lock_guard<std::mutex> lk(g_staging_mu);
    if ((int)g_staging.size() <= device) g_staging.resize(device + 1);
    if (!g_staging[device]) g_staging[device].reset(new Staging());
    return g_staging[device].get();
}

// Streams host keys through the staging buffers, calling launch(batch_on_device, first_key,
// buffer_index, stream) per chunk.  After the loop both streams are synchronized.
template <class Launch, class AfterChunk>
int pipeline_host_keys(Staging& st, const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
                       uint64_t n, int lp, bool need_out, Launch&& launch, AfterChunk&& after) {
    uint64_t lo = 0;
    int c = 0;
    uint64_t pending_lo[2] = {0, 0}, pending_n[2] = {0, 0};
    bool pending[2] = {false, false};
    while (lo < n) {
        // choose the chunk [lo, hi)
        uint64_t hi, bytes, base = 0;
        if (offsets) {
            // largest hi with offsets[hi] - offsets[lo] <= kChunkBytes (a single huge key alone)
            base = offsets[lo];
            const uint64_t* ub = std::upper_bound(offsets + lo + 1, offsets + n + 1, base + kChunkBytes);
            hi = (uint64_t)(ub - offsets) - 1;
            if (hi <= lo) hi = lo + 1;
            bytes = offsets[hi] - base;
        } else {
            uint64_t per = stride ? (kChunkBytes / stride) : n;
            if (per == 0) per = 1;
            hi = (n - lo) < per ? n : lo + per;
            bytes = (hi - lo) * stride;
        }
        const int b = c & 1;
        HIP_TRY(hipEventSynchronize(st.done[b]));  // buffer b free again
        if (pending[b]) {
            int rc = after(b, pending_lo[b], pending_n[b]);
            if (rc) return rc;
            pending[b] = false;
        }
        const uint8_t* src = keys + (offsets ? base : lo * stride);
        int rc;
        if (h2d_direct()) {
            // the runtime's own pageable path runs at the link rate: no host bounce copy
            rc = Staging::grow<uint8_t>(nullptr, &st.d_keys[b], &st.key_cap[b], bytes ? bytes : 1);
            if (rc) return rc;
            HIP_TRY(hipMemcpyAsync(st.d_keys[b], src, bytes, hipMemcpyHostToDevice, st.stream[b]));
        } else {
            rc = Staging::grow(&st.h_keys[b], &st.d_keys[b], &st.key_cap[b], bytes ? bytes : 1);
            if (rc) return rc;
            if (bytes) par_memcpy(st.h_keys[b], src, bytes);
            HIP_TRY(hipMemcpyAsync(st.d_keys[b], st.h_keys[b], bytes, hipMemcpyHostToDevice, st.stream[b]));
        }
        const uint64_t* d_off = nullptr;
        if (offsets) {
            rc = Staging::grow(&st.h_offs[b], &st.d_offs[b], &st.off_cap[b], hi - lo + 1);
            if (rc) return rc;
            par_memcpy(st.h_offs[b], offsets + lo, (hi - lo + 1) * sizeof(uint64_t));
            HIP_TRY(hipMemcpyAsync(st.d_offs[b], st.h_offs[b], (hi - lo + 1) * sizeof(uint64_t),
                                   hipMemcpyHostToDevice, st.stream[b]));
            d_off = st.d_offs[b];
        }
        if (need_out) {
            rc = Staging::grow(&st.h_out[b], &st.d_out[b], &st.out_cap[b], hi - lo);
            if (rc) return rc;
        }
        vbf::KeyBatch kb = batch(st.d_keys[b], d_off, base, stride, hi - lo, lp);
        rc = launch(kb, lo, b, st.stream[b]);
        if (rc) return rc;
        HIP_TRY(hipEventRecord(st.done[b], st.stream[b]));
        pending[b] = true;
        pending_lo[b] = lo;
        pending_n[b] = hi - lo;
        lo = hi;
        ++c;
    }
    for (int b = 0; b < 2; ++b) {
        HIP_TRY(hipStreamSynchronize(st.stream[b]));
        if (pending[b]) {
            int rc = after(b, pending_lo[b], pending_n[b]);
            if (rc) return rc;
            pending[b] = false;
        }
    }
    return VBF_OK;
}

// ---------------------------------------------------------------------------------------
// Filter handle.  Storage is shared between clones (bf.rs:249 clones the Arc).
// ---------------------------------------------------------------------------------------
struct Storage {
    int device = 0;  // VBF_DEVICE_HOST: the bits live in host memory (h_words), no HIP at all
    uint32_t m = 0;
    uint64_t nwords = 0;
    uint32_t* d_words = nullptr;
    // Host-resident bits.  Allocated on first use (host_words): a filter that is created on the
    // host and moved to a GPU before any set -- the compaction filter, bf.rs:62-81 then
    // build_filter_from_entries -- never zero-fills m/8 bytes of host memory.
    // Empty while pristine and never touched = all zero.
    std::vector<uint32_t> h_words;
    // The last asynchronous operation on d_words (a _dev call on the caller's stream): later
    // calls on other streams wait for it on the device, host-side calls wait for it on the host,
    // so every operation on one filter is ordered as the reference's Mutex<BitVec> orders them.
    hipEvent_t last = nullptr;
    bool pending = false;
    std::mutex mu;  // the reference's Mutex<BitVec>
    // Asynchronous set_host jobs (vbf_filter_set_host_async) queued on the device's worker and
    // not yet run.  Every other call on the filter first waits for them (storage_drain), so calls
    // stay ordered as the reference's Mutex orders them; a failed job's status is reported by the
    // next call that drains.
    uint64_t jobs_queued = 0, jobs_done = 0;
    pid_t jobs_pid = 0;  // the process whose worker runs the queued jobs (a forked child has none)
    std::condition_variable jobs_cv;
    int async_rc = VBF_OK;
    std::string async_msg;
    // Host mirror of d_words (device-resident filters only): a pinned copy that answers
    // single-key contains on the CPU, as the reference's read path calls it once per SST per get
    // (key_range/range.rs:130,136,171).  Valid while no device write happened since it was
    // filled; filled lazily by the first small contains (one D2H), or queued right after every
    // device write in VBF_MIRROR_EAGER mode.
    int mirror_mode = -1;  // -1: the process default (VBF_MIRROR, default lazy)
    // No bit was ever set since the array was created or cleared (BitVec::from_elem(m, false),
    // bf.rs:71): a migrate allocates zeroed words on the target instead of copying them.
    bool pristine = true;
    uint32_t* mirror = nullptr;
    bool mirror_ok = false;
    // vbf_filter_words_dev handed out d_words: a caller kernel may write the bits behind the
    // library's back, so the mirror is not trusted (every host read copies the words again) until
    // the caller declares its write with vbf_filter_stream_record.
    bool ext_write = false;
    bool mirror_current() const { return mirror_ok && !ext_write; }
    bool host() const { return device == VBF_DEVICE_HOST; }
    void free_mirror() {
        if (mirror && !hip_forked()) (void)hipHostFree(mirror);
        mirror = nullptr;
        mirror_ok = false;
    }
    ~Storage() {
        if (hip_forked()) {  // a forked child: the allocations are the parent's, and HIP is off limits
            mirror = nullptr;
            return;
        }
        if (d_words) {
            int prev = -1;
            (void)hipGetDevice(&prev);
            (void)hipSetDevice(device);
            if (pending) (void)hipEventSynchronize(last);
            (void)hipFree(d_words);
            if (prev >= 0) (void)hipSetDevice(prev);
        }
        free_mirror();
        if (last) (void)hipEventDestroy(last);
    }
};

// Caller holds s.mu, host-resident storage: the words, allocated (zeroed) on first use.
uint32_t* host_words(Storage& s) {
    if (s.h_words.size() != s.nwords) s.h_words.assign(s.nwords, 0u);
    return s.h_words.data();
}

// Caller holds s.mu: true when every queued asynchronous job has run.  Jobs queued by the parent
// of a forked child never run in the child (the worker thread stayed in the parent): the child
// counts them as failed instead of waiting for them forever.
bool storage_jobs_settled(Storage& s) {
    if (s.jobs_done == s.jobs_queued) return true;
    if (s.jobs_pid != getpid()) {
        s.jobs_done = s.jobs_queued;
        if (s.async_rc == VBF_OK) {
            s.async_rc = VBF_EINVAL;
            s.async_msg = "the process forked while an asynchronous set was queued; its bits are not in this copy";
        }
        return true;
    }
    return false;
}

// Caller holds `lk` on s.mu: waits until every asynchronous set_host job queued on the filter
// has run (the worker takes s.mu to run one, the wait releases it), then reports a failed job.
int storage_drain(Storage& s, std::unique_lock<std::mutex>& lk) {
    s.jobs_cv.wait(lk, [&] { return storage_jobs_settled(s); });
    if (s.async_rc != VBF_OK) {
        const int rc = s.async_rc;
        const std::string m = s.async_msg;
        s.async_rc = VBF_OK;
        s.async_msg.clear();
        return fail(rc, "an earlier asynchronous set on this filter failed: %s", m.c_str());
    }
    return VBF_OK;
}

int mirror_default() {
    static const int v = [] {
        const char* e = getenv("VBF_MIRROR");
        return e ? std::max(0, std::min(2, atoi(e))) : (int)VBF_MIRROR_LAZY;
    }();
    return v;
}
inline int mirror_mode(const Storage& s) { return s.mirror_mode < 0 ? mirror_default() : s.mirror_mode; }
// contains_host batches of at most this many keys answer from the mirror (~0.1 us per key on
// one core, against ~27 us for the staged GPU round trip)
uint64_t mirror_max_keys() {
    static const uint64_t v = [] {
        const char* e = getenv("VBF_MIRROR_MAX_KEYS");
        return e ? (uint64_t)strtoull(e, nullptr, 10) : (uint64_t)256;
    }();
    return v;
}

// Caller holds s.mu.  The stream `st` (any, including the legacy NULL stream) waits for the
// filter's last asynchronous operation.
int storage_wait(Storage& s, hipStream_t st) {
    if (s.pending) HIP_TRY(hipStreamWaitEvent(st, s.last, 0));
    return VBF_OK;
}
// Caller holds s.mu: the operation just queued on `st` is now the filter's last one.
int storage_mark(Storage& s, hipStream_t st) {
    if (!s.last) HIP_TRY(hipEventCreateWithFlags(&s.last, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(s.last, st));
    s.pending = true;
    return VBF_OK;
}
// Caller holds s.mu: the host waits until the filter's last asynchronous operation finished.
int storage_sync(Storage& s) {
    if (s.pending) {
        HIP_TRY(hipEventSynchronize(s.last));
        s.pending = false;
    }
    return VBF_OK;
}

// Caller holds s.mu, on s.device: a device write was just queued on `st` (and marked).  The
// mirror is stale; in eager mode its refresh is queued behind the write on the same stream, so
// it is valid once the filter's last event completes (every host reader syncs that first).
int mirror_after_write(Storage& s, hipStream_t st) {
    s.mirror_ok = false;
    if (mirror_mode(s) != VBF_MIRROR_EAGER || !s.nwords) return VBF_OK;
    if (!s.mirror) HIP_TRY(hipHostMalloc((void**)&s.mirror, s.nwords * 4, hipHostMallocDefault));
    HIP_TRY(hipMemcpyAsync(s.mirror, s.d_words, s.nwords * 4, hipMemcpyDeviceToHost, st));
    s.mirror_ok = true;
    return storage_mark(s, st);
}

// ---------------------------------------------------------------------------------------
// Host-resident filters (VBF_DEVICE_HOST): the memtable's filter, built one key per put
// (memtable/mem.rs:207-221: contains, then set) and probed one key per get (:223-230).  A GPU
// launch per key would cost two PCIe round trips per put, so these run on the CPU in the
// library, with the same SipHash-1-3 rounds as the kernels (sip13.hpp, compiled for the host)
// and Rust's `hash % m` (bf.rs:88,99).
// ---------------------------------------------------------------------------------------
vbf::Prefix host_prefix(const uint8_t* key, uint64_t len, bool lp) {
    vbf::Sip st = vbf::sip_init();
    if (lp) vbf::sip_compress(st, len);  // Hash for [u8]: write_usize(len) first
    uint64_t c = 0;
    for (; c + 8 <= len; c += 8) {
        uint64_t w;
        std::memcpy(&w, key + c, 8);  // little-endian block
        vbf::sip_compress(st, w);
    }
    vbf::Prefix p;
    p.st = st;
    p.r = (uint32_t)(len & 7);
    uint64_t t = 0;
    if (p.r) std::memcpy(&t, key + c, p.r);
    p.tail = t;
    p.total = (uint32_t)((len + (lp ? 8 : 0) + 8) & 0xff);
    return p;
}

inline void host_key(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t j,
                     const uint8_t** kp, uint64_t* len) {
    if (offsets) {
        *kp = keys + offsets[j];
        *len = offsets[j + 1] - offsets[j];
    } else {
        *kp = keys + j * stride;
        *len = stride;
    }
}

// bf.rs:84-92 per key (the caller counts the elements).
void host_set(uint32_t* w, uint32_t m, uint32_t k, const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
              uint64_t n, bool lp) {
    for (uint64_t j = 0; j < n; ++j) {
        const uint8_t* kp;
        uint64_t len;
        host_key(keys, offsets, stride, j, &kp, &len);
        const vbf::Prefix p = host_prefix(kp, len, lp);
        for (uint32_t i = 0; i < k; ++i) {
            const uint32_t idx = (uint32_t)(vbf::prefix_hash(p, i) % (uint64_t)m);
            w[idx >> 5] |= 1u << (idx & 31);
        }
    }
}

// bf.rs:95-105 per key: early exit on the first clear bit; k == 0 answers true.
void host_contains(const uint32_t* w, uint32_t m, uint32_t k, const uint8_t* keys, const uint64_t* offsets,
                   uint64_t stride, uint64_t n, bool lp, uint8_t* out) {
    for (uint64_t j = 0; j < n; ++j) {
        const uint8_t* kp;
        uint64_t len;
        host_key(keys, offsets, stride, j, &kp, &len);
        const vbf::Prefix p = host_prefix(kp, len, lp);
        uint8_t hit = 1;
        for (uint32_t i = 0; i < k; ++i) {
            const uint32_t idx = (uint32_t)(vbf::prefix_hash(p, i) % (uint64_t)m);
            if (!((w[idx >> 5] >> (idx & 31)) & 1u)) {
                hit = 0;
                break;
            }
        }
        out[j] = hit;
    }
}

std::mutex g_stream_mu;
std::vector<hipStream_t> g_filter_streams;

int filter_stream(int device, hipStream_t* out) {
    std::lock_guard<std::mutex> lk(g_stream_mu);
    if ((int)g_filter_streams.size() <= device) g_filter_streams.resize(device + 1, nullptr);
    if (!g_filter_streams[device]) HIP_TRY(hipStreamCreateWithFlags(&g_filter_streams[device], hipStreamNonBlocking));
    *out = g_filter_streams[device];
    return VBF_OK;
}

// Caller holds s.mu (drained), on s.device: the mirror holds the current bits (one D2H when
// it is stale).
int mirror_fill(Storage& s) {
    int rc = storage_sync(s);
    if (rc) return rc;
    if (s.mirror_current() || !s.nwords) return VBF_OK;
    if (!s.mirror) HIP_TRY(hipHostMalloc((void**)&s.mirror, s.nwords * 4, hipHostMallocDefault));
    hipStream_t fs;
    if ((rc = filter_stream(s.device, &fs))) return rc;
    HIP_TRY(hipMemcpyAsync(s.mirror, s.d_words, s.nwords * 4, hipMemcpyDeviceToHost, fs));
    HIP_TRY(hipStreamSynchronize(fs));
    s.mirror_ok = true;
    return VBF_OK;
}

int new_storage(int device, uint32_t m, std::shared_ptr<Storage>* out) {
    auto s = std::make_shared<Storage>();
    s->device = device;
    s->m = m;
    s->nwords = ((uint64_t)m + 31) / 32;
    if (device == VBF_DEVICE_HOST) {
        // BitVec::from_elem(m, false) (bf.rs:71): allocated on first use (host_words)
    } else if (s->nwords) {
        hipStream_t st;
        int rc = filter_stream(device, &st);
        if (rc) return rc;
        HIP_TRY(hipMalloc((void**)&s->d_words, s->nwords * 4));
        // zeroed on the filter's stream, not waited for: every later use of the words is ordered
        // after the filter's last event (storage_wait / storage_sync)
        HIP_TRY(hipMemsetAsync(s->d_words, 0, s->nwords * 4, st));
        if ((rc = storage_mark(*s, st))) return rc;
    }
    *out = std::move(s);
    return VBF_OK;
}

// ---------------------------------------------------------------------------------------
// Phase profiling: when enabled, every kernel phase is bracketed by hipEvents on its stream.
// ---------------------------------------------------------------------------------------
std::atomic<bool> g_prof{false};
std::mutex g_prof_mu;
struct PhaseRec {
    int phase;
    hipEvent_t a, b;
};
std::vector<PhaseRec> g_prof_recs;
thread_local hipEvent_t g_open[vbf::kNumPhases] = {};

}  // namespace

namespace vbf {
void phase_begin(int phase, hipStream_t s) {
    if (!g_prof.load(std::memory_order_relaxed)) return;
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    (void)hipEventRecord(e, s);
    g_open[phase] = e;
}
void phase_end(int phase, hipStream_t s) {
    if (!g_prof.load(std::memory_order_relaxed) || !g_open[phase]) return;
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    (void)hipEventRecord(e, s);
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_recs.push_back(PhaseRec{phase, g_open[phase], e});
    g_open[phase] = nullptr;
}
}  // namespace vbf

namespace {

// ---------------------------------------------------------------------------------------
// SST data.db decode (vbf_sst.hip): count pass + scan, one 16-byte readback (entry total and
// error word) so the caller can size or validate, then the emit pass queued on the stream.
// ---------------------------------------------------------------------------------------
inline uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }

int sst_count_pass(const uint8_t* data, uint64_t len, const uint32_t* blocks, uint64_t nblocks,
                   hipStream_t s, vbf::SstArgs* a, uint64_t* n_out, uint32_t* uniform_len = nullptr) {
    *a = vbf::SstArgs{};
    *n_out = 0;
    if (uniform_len) *uniform_len = 0xFFFFFFFFu;
    if (len && (!data || !blocks || !nblocks))
        return fail(VBF_EINVAL, "data.db of %llu bytes needs its block start offsets (index.db)",
                    (unsigned long long)len);
    if (!len && nblocks) return fail(VBF_EINVAL, "%llu block offsets for an empty data.db", (unsigned long long)nblocks);
    if (nblocks >= 0x7FFFFFFFull) return fail(VBF_EINVAL, "too many blocks (%llu)", (unsigned long long)nblocks);
    if (!len) return VBF_OK;
    size_t tmpb = 0, tmpr = 0;
    HIP_TRY(vbf::sst_scan(nullptr, nullptr, nblocks + 1, nullptr, &tmpb, s));
    HIP_TRY(vbf::sst_len_range(nullptr, nullptr, nblocks, nullptr, nullptr, &tmpr, s));
    tmpb = std::max(tmpb, tmpr);
    const uint64_t o_ebase = align256((nblocks + 1) * 4);
    const uint64_t o_pos = o_ebase + align256((nblocks + 1) * 8);
    const uint64_t o_lmin = o_pos + align256(vbf::sst_pos_bytes(nblocks));
    const uint64_t o_lmax = o_lmin + align256(nblocks * 4);
    const uint64_t o_err = o_lmax + align256(nblocks * 4);
    const uint64_t o_tmp = o_err + 256;
    void* ws = nullptr;
    int rc = get_workspace(s, o_tmp + tmpb, &ws, kWsSstScratch);
    if (rc) return rc;
    char* base = static_cast<char*>(ws);
    uint32_t* counts = reinterpret_cast<uint32_t*>(base);
    uint64_t* ebase = reinterpret_cast<uint64_t*>(base + o_ebase);
    uint32_t* err = reinterpret_cast<uint32_t*>(base + o_err);
    HIP_TRY(hipMemsetAsync(counts, 0, (nblocks + 1) * 4, s));
    HIP_TRY(hipMemsetAsync(err, 0, 4, s));
    HIP_TRY(hipMemsetAsync(err + 1, 0xFF, 12, s));
    uint16_t* pos = reinterpret_cast<uint16_t*>(base + o_pos);
    static const uint32_t walk_v = [] {  // VBF_SST_WALK=0: the scalar entry walk (A/B)
        const char* e = getenv("VBF_SST_WALK");
        return e ? (uint32_t)(atoi(e) != 0) : 1u;
    }();
    static const uint32_t abl = [] {
        const char* e = VBF_ABLATION_BUILD ? getenv("VBF_ABLATE") : nullptr;
        return e ? (uint32_t)atoi(e) : 0u;
    }();
    uint32_t* lmin = reinterpret_cast<uint32_t*>(base + o_lmin);
    uint32_t* lmax = reinterpret_cast<uint32_t*>(base + o_lmax);
    *a = vbf::SstArgs{data, len, blocks, nblocks, counts, pos, lmin, lmax, ebase, nullptr, nullptr, nullptr, nullptr,
                      nullptr, err, abl, walk_v};
    vbf::phase_begin(vbf::kPhaseSstWalk, s);
    HIP_TRY(vbf::sst_count(*a, s));
    vbf::phase_end(vbf::kPhaseSstWalk, s);
    vbf::phase_begin(vbf::kPhaseSstScan, s);
    HIP_TRY(vbf::sst_scan(counts, ebase, nblocks + 1, base + o_tmp, &tmpb, s));
    if (uniform_len) HIP_TRY(vbf::sst_len_range(lmin, lmax, nblocks, err + 2, base + o_tmp, &tmpb, s));
    vbf::phase_end(vbf::kPhaseSstScan, s);
    uint64_t total = 0;
    uint32_t ev[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(&total, ebase + nblocks, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(ev, err, 16, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (ev[0]) {
        const char* what = (ev[0] & 8) ? "block offsets not increasing / not starting at 0 / past the end"
                         : (ev[0] & 4) ? "block larger than 65535 bytes"
                         : (ev[0] & 2) ? "more than 256 entries in a block"
                                       : "entry crosses the block end (truncated data.db or wrong index)";
        return fail(VBF_EINVAL, "malformed data.db at block %u: %s", ev[1], what);
    }
    if (len < 17 * total) return fail(VBF_EINVAL, "inconsistent entry count %llu", (unsigned long long)total);
    *n_out = total;
    if (uniform_len && total && ev[2] == ev[3] && a->ablate == 0) *uniform_len = ev[2];
    return VBF_OK;
}

int sst_emit_pass(vbf::SstArgs a, uint8_t* keys, uint64_t* offsets, uint32_t* val_off, uint64_t* created,
                  uint8_t* tomb, hipStream_t s) {
    if (!a.len) {
        if (offsets) HIP_TRY(hipMemsetAsync(offsets, 0, 8, s));
        return VBF_OK;
    }
    if (keys && ((uintptr_t)keys & 3)) return fail(VBF_EINVAL, "keys buffer must be 4-byte aligned");
    a.keys = keys;
    a.offsets = offsets;
    a.val_off = val_off;
    a.created = created;
    a.tomb = tomb;
    if (!keys && !offsets && !val_off && !created && !tomb) return VBF_OK;
    vbf::phase_begin(vbf::kPhaseSstEmit, s);
    HIP_TRY(vbf::sst_emit(a, s));
    vbf::phase_end(vbf::kPhaseSstEmit, s);
    return VBF_OK;
}

// index.db (indexer.rs:151-170: u32 key_len | key | u32 block offset per block) -> offsets.
int parse_index(const uint8_t* index, uint64_t len, std::vector<uint32_t>* out) {
    out->clear();
    uint64_t p = 0;
    while (p < len) {
        if (len - p < 4) return fail(VBF_EINVAL, "index.db truncated at byte %llu", (unsigned long long)p);
        uint32_t L;
        memcpy(&L, index + p, 4);
        if (len - p - 4 < (uint64_t)L + 4) return fail(VBF_EINVAL, "index.db truncated at byte %llu", (unsigned long long)p);
        uint32_t off;
        memcpy(&off, index + p + 4 + L, 4);
        out->push_back(off);
        p += (uint64_t)L + 8;
    }
    return VBF_OK;
}

// ---------------------------------------------------------------------------------------
// Host keys into a device-resident filter.  Caller holds s.mu (drained), on s.device: the keys
// stream through the device's staging pipeline (H2D of chunk c+1 under the kernels of chunk c)
// and the bits are merged into d_words; returns with the work finished.
// ---------------------------------------------------------------------------------------
int device_set_host(Storage& s, uint32_t k, const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
                    uint64_t n, int lp) {
    Staging* st = staging_for(s.device);
    std::lock_guard<std::mutex> lk2(st->mu);
    int rc = st->init(s.device);
    if (rc) return rc;
    if ((rc = storage_sync(s))) return rc;  // earlier _dev work on this filter, any stream
    s.mirror_ok = false;
    // A pristine filter (new or cleared, never written: the compaction filter, sized.rs:192-193)
    // takes its first chunk as BloomFilter::new fused with the build (VBF_BUILD_FRESH: the segment
    // pass writes its words without reading them, where one chunk and one workgroup per segment
    // allow), as the benchmark's step does; the other chunks wait for it on the device, then OR
    // in with word atomics as before.
    const bool fresh = s.pristine;
    s.pristine = false;
    rc = pipeline_host_keys(
        *st, keys, offsets, stride, n, lp, false,
        [&](const vbf::KeyBatch& kb, uint64_t lo, int, hipStream_t hs) -> int {
            if (fresh && lo == 0) {
                int r = do_build(kb, s.m, k, s.d_words, VBF_BUILD_AUTO | VBF_BUILD_FRESH, false, hs);
                if (r) return r;
                HIP_TRY(hipEventRecord(st->first, hs));
                return VBF_OK;
            }
            if (fresh) HIP_TRY(hipStreamWaitEvent(hs, st->first, 0));
            return do_build(kb, s.m, k, s.d_words, VBF_BUILD_AUTO, true, hs);
        },
        [](int, uint64_t, uint64_t) { return VBF_OK; });
    if (rc) return rc;
    return mirror_after_write(s, st->stream[0]);
}

// ---------------------------------------------------------------------------------------
// Asynchronous set_host (vbf_filter_set_host_async): one worker thread per device runs the
// queued jobs in order, each exactly as a synchronous set_host would under the filter's lock.
// The submitting thread returns at once, so a serial caller -- the compaction loop that builds
// one filter per merged table (compactors/sized.rs:170-200) -- keeps merging the next table
// while the GPUs build, one filter per device with VBF_DEVICE_AUTO placement.
// ---------------------------------------------------------------------------------------
struct AsyncJob {
    std::shared_ptr<Storage> s;
    uint32_t k = 0;
    const uint8_t* keys = nullptr;
    const uint64_t* offsets = nullptr;
    uint64_t stride = 0, n = 0;
    int lp = 1;
    std::unique_ptr<uint8_t[]> own_keys;  // the library's copy when the caller passed no release
    std::unique_ptr<uint64_t[]> own_offs;
    void (*release)(void*) = nullptr;
    void* ctx = nullptr;
};

class AsyncQueue {
  public:
    static AsyncQueue& get(int device) {
        static std::mutex mu;
        static std::vector<AsyncQueue*> qs;  // never destroyed: the workers outlive static teardown
        std::lock_guard<std::mutex> lk(mu);
        if ((int)qs.size() <= device) qs.resize(device + 1, nullptr);
        // a forked child inherits the queue objects but not their threads: start new ones
        if (!qs[device] || qs[device]->pid_ != getpid()) qs[device] = new AsyncQueue();
        return *qs[device];
    }
    void push(AsyncJob* j) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(j);
        }
        cv_.notify_one();
    }

  private:
    AsyncQueue() : pid_(getpid()) { std::thread([this] { loop(); }).detach(); }
    void loop() {
        for (;;) {
            AsyncJob* j;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return !q_.empty(); });
                j = q_.front();
                q_.erase(q_.begin());
            }
            run(*j);
            Storage& s = *j->s;
            {
                std::lock_guard<std::mutex> lk(s.mu);
                ++s.jobs_done;
            }
            s.jobs_cv.notify_all();
            // after the job counts as done: a release callback may call back into the library
            // (vbf_filter_sync, or a free in a Rust Drop) without waiting for its own job
            if (j->release) j->release(j->ctx);
            delete j;
        }
    }
    static void run(AsyncJob& j) {
        Storage& s = *j.s;
        std::lock_guard<std::mutex> lk(s.mu);
        int rc;
        {
            DeviceGuard g(s.device);
            if (g.forked) {
                rc = fail_forked();
            } else if (g.err != hipSuccess) {
                rc = fail(VBF_ENODEV, "hipSetDevice(%d): %s", s.device, hipGetErrorString(g.err));
            } else {
                (void)hipGetLastError();  // no earlier job's failure is this job's
                rc = device_set_host(s, j.k, j.keys, j.offsets, j.stride, j.n, j.lp);
            }
        }
        if (rc && s.async_rc == VBF_OK) {  // the first failure is reported by the next call that drains
            s.async_rc = rc;
            s.async_msg = g_err;
        }
    }
    const pid_t pid_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<AsyncJob*> q_;
};

std::atomic<uint64_t> g_auto_rr{0};

// xor over words of (w_i * G + (i + 1) * C), 64-bit wrapping: velarixdb_amd/filter_file.py's
// fast_checksum, the integrity word of the persisted bit array.
uint64_t words_checksum(const uint32_t* w, uint64_t nwords) {
    constexpr uint64_t G = 0x9E3779B97F4A7C15ull, C = 0xC2B2AE3D27D4EB4Full;
    CopyPool& pool = CopyPool::get();
    const unsigned nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(pool.threads(), nwords >> 20));
    std::vector<uint64_t> part(nt, 0);
    auto body = [&](unsigned t) {
        const uint64_t a = nwords * t / nt, b = nwords * (t + 1) / nt;
        uint64_t x = 0;
        for (uint64_t i = a; i < b; ++i) x ^= (uint64_t)w[i] * G + (i + 1) * C;
        part[t] = x;
    };
    if (nt == 1) body(0);
    else pool.run(nt, body);
    uint64_t x = 0;
    for (uint64_t v : part) x ^= v;
    return x;
}

}  // namespace

struct vbf_filter {
    std::shared_ptr<Storage> bits;
    uint32_t k = 0;
    std::atomic<uint32_t> n{0};
    double p = 0.0;
    // Binding bookkeeping that lives in the handle, so a binding's BloomFilter needs no private
    // fields (velarixdb builds `BloomFilter { file_path, ..Default::default() }` outside
    // filter::bf: db/recovery.rs:143-146, tests/workload.rs:309-312).  Per handle, copied by clone
    // like the struct's other plain fields (bf.rs:242-254).
    std::atomic<uint64_t> sst_entries{VBF_EXT_NONE};  // the SST's entry count (build_filter_from_entries)
    std::atomic<int> restored{0};  // vbf_filter_recover_ext loaded persisted bits (not yet taken)
};

extern "C" {

const char* vbf_version(void) { return "velarixdb_amd-vbf 0.2.0 gfx950"; }

int vbf_profile_enable(int on) {
    g_prof.store(on != 0);
    return ok();
}

int vbf_profile_read(double* ms, uint64_t* launches, int nphases) {
    FORK_GUARD();
    if (!ms || !launches || nphases < 0) return fail(VBF_EINVAL, "NULL argument");
    for (int i = 0; i < nphases; ++i) {
        ms[i] = 0.0;
        launches[i] = 0;
    }
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (auto& r : g_prof_recs) {
        float t = 0.f;
        HIP_TRY(hipEventSynchronize(r.b));
        HIP_TRY(hipEventElapsedTime(&t, r.a, r.b));
        if (r.phase < nphases) {
            ms[r.phase] += t;
            launches[r.phase] += 1;
        }
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    g_prof_recs.clear();
    return ok();
}

const char* vbf_last_error(void) { return g_err.c_str(); }

int vbf_device_count(int* count) {
    if (!count) return fail(VBF_EINVAL, "count is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *count = 0;
        return fail(VBF_ENODEV, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *count = c;
    return ok();
}

uint32_t vbf_num_bits(uint64_t n, double p) {
    const double ln2 = std::log(2.0);
    const double x = ((double)n * std::log(p)) / (ln2 * ln2);  // powi(2) == one multiply
    return f64_as_u32(-std::ceil(x));
}

uint32_t vbf_num_hash_functions(uint32_t m, uint32_t n) {
    const double x = ((double)m / (double)n) * std::ceil(std::log(2.0));  // ln2.ceil() == 1
    return f64_as_u32(x);
}

int vbf_size(double p, uint64_t n, uint32_t* m, uint32_t* k) {
    if (!m || !k) return fail(VBF_EINVAL, "NULL output");
    if (!(p >= 0.0)) return fail(VBF_EINVAL, "False positive rate can not be less than or equal to zero");
    if (n == 0) return fail(VBF_EINVAL, "No of elements should be greater than 0");
    *m = vbf_num_bits(n, p);
    *k = vbf_num_hash_functions(*m, (uint32_t)n);
    return ok();
}

void vbf_meta_serialize(uint32_t k, uint32_t n, double p, uint8_t out[16]) {
    uint64_t pb;
    std::memcpy(&pb, &p, 8);
    for (int i = 0; i < 4; ++i) out[i] = (uint8_t)(k >> (8 * i));
    for (int i = 0; i < 4; ++i) out[4 + i] = (uint8_t)(n >> (8 * i));
    for (int i = 0; i < 8; ++i) out[8 + i] = (uint8_t)(pb >> (8 * i));
}

int vbf_meta_parse(const uint8_t* in, size_t len, uint32_t* k, uint32_t* n, double* p) {
    if (!in || !k || !n || !p) return fail(VBF_EINVAL, "NULL argument");
    if (len < 16) return fail(VBF_EINVAL, "filter metadata truncated: %zu < 16 bytes (unexpected EOF)", len);
    uint32_t kk = 0, nn = 0;
    uint64_t pb = 0;
    for (int i = 3; i >= 0; --i) kk = (kk << 8) | in[i];
    for (int i = 3; i >= 0; --i) nn = (nn << 8) | in[4 + i];
    for (int i = 7; i >= 0; --i) pb = (pb << 8) | in[8 + i];
    *k = kk;
    *n = nn;
    std::memcpy(p, &pb, 8);
    return ok();
}

// ---- stateless device-pointer entry points ----

int vbf_build_dev(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                  int len_prefix, uint32_t m, uint32_t k, uint32_t* words, void* stream) {
    return vbf_build_dev_ex(keys, offsets, stride, n, len_prefix, m, k, words, VBF_BUILD_AUTO, stream);
}

uint64_t vbf_build_workspace_bytes(uint64_t n, uint32_t m, uint32_t k) {
    return vbf::partition_workspace_bytes(n, m, k);
}

int vbf_release_workspaces(void) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    if (hip_forked()) {  // the parent's buffers: forget them, free nothing
        g_ws.clear();
        return ok();
    }
    for (auto& w : g_ws) {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(w.device);
        (void)hipStreamSynchronize(w.stream);
        (void)hipFree(w.ptr);
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    g_ws.clear();
    return ok();
}

int vbf_build_dev_ex(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                     int len_prefix, uint32_t m, uint32_t k, uint32_t* words, int strategy, void* stream) {
    FORK_GUARD();
    int rc = check_mk(m, k, n);
    if (rc) return rc;
    if ((rc = check_keys(keys, offsets, stride, n))) return rc;
    if (n && k && !words) return fail(VBF_EINVAL, "words is NULL");
    vbf::KeyBatch kb = batch(keys, offsets, 0, stride, n, len_prefix);
    if ((rc = do_build(kb, m, k, words, strategy, false, (hipStream_t)stream))) return rc;
    return ok();
}

int vbf_probe_dev_ex(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                     int len_prefix, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
                     int strategy, void* stream) {
    FORK_GUARD();
    int rc = check_mk(m, k, n);
    if (rc) return rc;
    if ((rc = check_keys(keys, offsets, stride, n))) return rc;
    if (n && !out) return fail(VBF_EINVAL, "out is NULL");
    vbf::KeyBatch kb = batch(keys, offsets, 0, stride, n, len_prefix);
    if ((rc = do_probe(kb, m, k, words, out, nullptr, strategy, (hipStream_t)stream))) return rc;
    return ok();
}

int vbf_probe_dev(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                  int len_prefix, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
                  void* stream) {
    return vbf_probe_dev_ex(keys, offsets, stride, n, len_prefix, m, k, words, out, VBF_BUILD_AUTO, stream);
}

int vbf_probe_count_dev_ex(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                           int len_prefix, uint32_t m, uint32_t k, const uint32_t* words,
                           unsigned long long* count_dev, int strategy, void* stream) {
    FORK_GUARD();
    int rc = check_mk(m, k, n);
    if (rc) return rc;
    if ((rc = check_keys(keys, offsets, stride, n))) return rc;
    if (!count_dev) return fail(VBF_EINVAL, "count_dev is NULL");
    vbf::KeyBatch kb = batch(keys, offsets, 0, stride, n, len_prefix);
    if ((rc = do_probe(kb, m, k, words, nullptr, count_dev, strategy, (hipStream_t)stream))) return rc;
    return ok();
}

int vbf_probe_count_dev(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                        int len_prefix, uint32_t m, uint32_t k, const uint32_t* words,
                        unsigned long long* count_dev, void* stream) {
    return vbf_probe_count_dev_ex(keys, offsets, stride, n, len_prefix, m, k, words, count_dev, VBF_BUILD_AUTO,
                                  stream);
}

int vbf_hashes_dev(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                   int len_prefix, uint32_t k, uint64_t* out, void* stream) {
    FORK_GUARD();
    int rc = check_keys(keys, offsets, stride, n);
    if (rc) return rc;
    if (n && k && !out) return fail(VBF_EINVAL, "out is NULL");
    vbf::KeyBatch kb = batch(keys, offsets, 0, stride, n, len_prefix);
    HIP_TRY(vbf::launch_hashes(kb, k, out, (hipStream_t)stream));
    return ok();
}

int vbf_or_words_dev(uint32_t* dst, const uint32_t* src, uint64_t nwords, void* stream) {
    FORK_GUARD();
    if (nwords && (!dst || !src)) return fail(VBF_EINVAL, "NULL words");
    HIP_TRY(vbf::launch_or_words(dst, src, nwords, (hipStream_t)stream));
    return ok();
}

extern "C++" {
namespace vbf {  // vbf_kernels.hip
hipError_t launch_or_fold(uint32_t* dst, const uint32_t* src, uint64_t nwords, uint32_t parts, uint64_t pstride,
                          hipStream_t s);
}
}

int vbf_or_fold_dev(uint32_t* dst, const uint32_t* src, uint64_t nwords, uint32_t nparts, uint64_t part_stride,
                    void* stream) {
    FORK_GUARD();
    if (nwords && nparts && (!dst || !src)) return fail(VBF_EINVAL, "NULL words");
    if (nparts > 1 && part_stride < nwords) return fail(VBF_EINVAL, "parts overlap (stride %llu < %llu words)",
                                                        (unsigned long long)part_stride, (unsigned long long)nwords);
    const hipError_t e = vbf::launch_or_fold(dst, src, nwords, nparts, part_stride, (hipStream_t)stream);
    if (e == hipErrorInvalidValue) return fail(VBF_EINVAL, "vbf_or_fold_dev needs 16-byte aligned words and a stride of whole 4-word units");
    HIP_TRY(e);
    return ok();
}

int vbf_popcount_dev(const uint32_t* words, uint64_t nwords, unsigned long long* count_dev, void* stream) {
    FORK_GUARD();
    if (!count_dev || (nwords && !words)) return fail(VBF_EINVAL, "NULL argument");
    HIP_TRY(vbf::launch_popcount(words, nwords, count_dev, (hipStream_t)stream));
    return ok();
}

int vbf_gen_fixed_dev(uint64_t seed, uint64_t base, uint64_t n, uint32_t len, uint8_t* out, void* stream) {
    FORK_GUARD();
    if (n && len && !out) return fail(VBF_EINVAL, "out is NULL");
    HIP_TRY(vbf::launch_gen_fixed(seed, base, n, len, out, (hipStream_t)stream));
    return ok();
}

int vbf_gen_var_dev(uint64_t seed, uint64_t base, uint64_t n, const uint64_t* offsets, uint8_t* out,
                    void* stream) {
    FORK_GUARD();
    if (n && (!offsets || !out)) return fail(VBF_EINVAL, "NULL argument");
    HIP_TRY(vbf::launch_gen_var(seed, base, n, offsets, out, (hipStream_t)stream));
    return ok();
}

int vbf_gen_sst_fixed_dev(uint64_t seed, uint64_t base, uint64_t n, uint32_t len, uint8_t* data,
                          uint32_t* blocks, void* stream) {
    FORK_GUARD();
    if (n && (!data || !blocks)) return fail(VBF_EINVAL, "NULL argument");
    if (len + 17 > 4096) return fail(VBF_EINVAL, "an entry of %u + 17 bytes exceeds a 4096-byte block", len);
    HIP_TRY(vbf::gen_sst_fixed(seed, base, n, len, data, blocks, (hipStream_t)stream));
    return ok();
}

// ---- one-shot host-pointer entry points ----

int vbf_build_host(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                   int len_prefix, uint32_t m, uint32_t k, uint32_t* words, uint64_t nwords,
                   int device) {
    int rc = check_mk(m, k, n);
    if (rc) return rc;
    if ((rc = check_keys(keys, offsets, stride, n))) return rc;
    const uint64_t need = ((uint64_t)m + 31) / 32;
    if (nwords < need || (need && !words)) return fail(VBF_EINVAL, "words holds %llu < ceil(m/32) = %llu",
                                                       (unsigned long long)nwords, (unsigned long long)need);
    if (n == 0 || k == 0) return ok();
    DEVICE_SCOPE(device);
    Staging* st = staging_for(device);
    std::lock_guard<std::mutex> lk(st->mu);
    if ((rc = st->init(device))) return rc;
    if ((rc = Staging::grow<uint32_t>(nullptr, &st->d_words, &st->words_cap, need))) return rc;
    if ((rc = xfer_h2d(*st, st->d_words, words, need * 4))) return rc;
    rc = pipeline_host_keys(
        *st, keys, offsets, stride, n, len_prefix, false,
        [&](const vbf::KeyBatch& kb, uint64_t, int, hipStream_t s) -> int {
            return do_build(kb, m, k, st->d_words, VBF_BUILD_AUTO, true, s);
        },
        [](int, uint64_t, uint64_t) { return VBF_OK; });
    if (rc) return rc;
    if ((rc = xfer_d2h(*st, words, st->d_words, need * 4))) return rc;
    return ok();
}

int vbf_build_shards_host(vbf_shard* shards, uint64_t nshards, const int* devices, int ndevices) {
    if (nshards && !shards) return fail(VBF_EINVAL, "shards is NULL");
    if (nshards && (!devices || ndevices <= 0)) return fail(VBF_EINVAL, "no devices given");
    std::vector<std::string> msg(nshards);
    auto work = [&](int d) {
        for (uint64_t s = (uint64_t)d; s < nshards; s += (uint64_t)ndevices) {
            vbf_shard& sh = shards[s];
            sh.status = vbf_build_host(sh.keys, sh.offsets, sh.stride, sh.n, sh.len_prefix, sh.m, sh.k, sh.words,
                                       sh.nwords, devices[d]);
            if (sh.status) msg[s] = g_err;
        }
    };
    const int nt = (int)std::min<uint64_t>((uint64_t)ndevices, nshards);
    std::vector<std::thread> th;
    th.reserve(nt > 0 ? nt - 1 : 0);
    for (int d = 1; d < nt; ++d) th.emplace_back(work, d);
    if (nt > 0) work(0);
    for (auto& t : th) t.join();
    for (uint64_t s = 0; s < nshards; ++s)
        if (shards[s].status) return fail(shards[s].status, "shard %llu: %s", (unsigned long long)s, msg[s].c_str());
    return ok();
}

int vbf_probe_host(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                   int len_prefix, uint32_t m, uint32_t k, const uint32_t* words, uint64_t nwords,
                   uint8_t* out, int device) {
    int rc = check_mk(m, k, n);
    if (rc) return rc;
    if ((rc = check_keys(keys, offsets, stride, n))) return rc;
    const uint64_t need = ((uint64_t)m + 31) / 32;
    if (nwords < need || (need && !words)) return fail(VBF_EINVAL, "words too short");
    if (n && !out) return fail(VBF_EINVAL, "out is NULL");
    if (n == 0) return ok();
    DEVICE_SCOPE(device);
    Staging* st = staging_for(device);
    std::lock_guard<std::mutex> lk(st->mu);
    if ((rc = st->init(device))) return rc;
    if ((rc = Staging::grow<uint32_t>(nullptr, &st->d_words, &st->words_cap, need ? need : 1))) return rc;
    if (need) HIP_TRY(hipMemcpyAsync(st->d_words, words, need * 4, hipMemcpyHostToDevice, st->stream[0]));
    HIP_TRY(hipEventRecord(st->done[0], st->stream[0]));
    HIP_TRY(hipStreamWaitEvent(st->stream[1], st->done[0], 0));
    rc = pipeline_host_keys(
        *st, keys, offsets, stride, n, len_prefix, true,
        [&](const vbf::KeyBatch& kb, uint64_t, int b, hipStream_t s) -> int {
            if (int rc2 = do_probe(kb, m, k, st->d_words, st->d_out[b], nullptr, VBF_BUILD_AUTO, s)) return rc2;
            HIP_TRY(hipMemcpyAsync(st->h_out[b], st->d_out[b], kb.n, hipMemcpyDeviceToHost, s));
            return VBF_OK;
        },
        [&](int b, uint64_t lo, uint64_t cnt) {
            par_memcpy(out + lo, st->h_out[b], cnt);
            return VBF_OK;
        });
    if (rc) return rc;
    return ok();
}

// ---- filter handle ----
//
// Every entry point takes the filter's lock (Storage::mu, the reference's Mutex<BitVec>) BEFORE
// it looks at where the bits live: vbf_filter_migrate changes device / d_words / h_words under
// that lock and clones share the Storage, so a residency read outside it could send a call down
// the wrong path.  Then it drains the filter's queued asynchronous sets (storage_drain).

static int make_filter(int device, uint32_t m, uint32_t k, double p, vbf_filter** out) {
    if (!out) return fail(VBF_EINVAL, "out is NULL");
    std::unique_ptr<vbf_filter> f(new vbf_filter());
    if (device == VBF_DEVICE_HOST) {
        int rc = new_storage(device, m, &f->bits);
        if (rc) return rc;
    } else {
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
            return fail(VBF_ENODEV, "no HIP device available");
        // placement policy: filters created with VBF_DEVICE_AUTO go round-robin over the devices,
        // so one serial caller's successive filters (one per merged table) land on different GPUs
        if (device == VBF_DEVICE_AUTO) device = (int)(g_auto_rr.fetch_add(1) % (uint64_t)count);
        if (device < 0 || device >= count)
            return fail(VBF_ENODEV, "device %d out of range (%d devices)", device, count);
        DEVICE_SCOPE(device);
        int rc = new_storage(device, m, &f->bits);
        if (rc) return rc;
    }
    f->k = k;
    f->p = p;
    *out = f.release();
    return ok();
}

static int host_resident(const char* what) {
    return fail(VBF_EINVAL, "%s: the filter is host-resident (VBF_DEVICE_HOST); use the _host entry points", what);
}

int vbf_filter_new(double p, uint64_t no_of_elements, int device, vbf_filter** out) {
    uint32_t m, k;
    int rc = vbf_size(p, no_of_elements, &m, &k);
    if (rc) return rc;
    return make_filter(device, m, k, p, out);
}

int vbf_filter_default(int device, vbf_filter** out) { return make_filter(device, 0, 0, 0.0, out); }

int vbf_filter_new_sized(uint32_t m, uint32_t k, double p, int device, vbf_filter** out) {
    return make_filter(device, m, k, p, out);
}

int vbf_filter_recover(const uint8_t* meta, size_t len, int device, vbf_filter** out) {
    uint32_t k, n;
    double p;
    int rc = vbf_meta_parse(meta, len, &k, &n, &p);
    if (rc) return rc;
    // bf.rs:144-147: m is recomputed from the STORED element count (usize) and p.
    rc = make_filter(device, vbf_num_bits((uint64_t)n, p), k, p, out);
    if (rc) return rc;
    (*out)->n.store(n);
    return ok();
}

int vbf_filter_clone(const vbf_filter* f, vbf_filter** out) {
    if (!f || !out) return fail(VBF_EINVAL, "NULL argument");
    vbf_filter* c = new vbf_filter();
    c->bits = f->bits;
    c->k = f->k;
    c->n.store(f->n.load());  // bf.rs:248: the clone's counter is a copy, the bits are shared
    c->p = f->p;
    c->sst_entries.store(f->sst_entries.load());
    c->restored.store(f->restored.load());
    *out = c;
    return ok();
}

void vbf_filter_free(vbf_filter* f) { delete f; }

uint32_t vbf_filter_num_bits(const vbf_filter* f) { return f ? f->bits->m : 0; }
uint32_t vbf_filter_num_elements(const vbf_filter* f) { return f ? f->n.load() : 0; }
uint32_t vbf_filter_num_hash_functions(const vbf_filter* f) { return f ? f->k : 0; }
double vbf_filter_false_positive_rate(const vbf_filter* f) { return f ? f->p : 0.0; }
int vbf_filter_device(const vbf_filter* f) {
    if (!f) return VBF_DEVICE_HOST - 1;
    std::lock_guard<std::mutex> lk(f->bits->mu);
    return f->bits->device;
}
uint64_t vbf_filter_host_bytes(const vbf_filter* f) {
    if (!f) return 0;
    Storage& s = *f->bits;
    std::lock_guard<std::mutex> lk(s.mu);
    return (uint64_t)s.h_words.size() * 4 + (s.mirror ? s.nwords * 4 : 0);
}

uint32_t* vbf_filter_words_dev(const vbf_filter* f) {
    if (!f) return nullptr;
    Storage& s = *f->bits;
    std::lock_guard<std::mutex> lk(s.mu);
    // the caller's kernels are not ordered after the filter's last event (e.g. the asynchronous
    // zeroing of a new filter's words): wait for it here
    if (!hip_forked() && storage_sync(s) != VBF_OK) return nullptr;
    if (s.d_words) {
        // the caller may write through the pointer: the bits are no longer known to be zero, and
        // the host mirror is bypassed until the write is declared (vbf_filter_stream_record)
        s.pristine = false;
        s.mirror_ok = false;
        s.ext_write = true;
    }
    return s.d_words;
}

const uint32_t* vbf_filter_words_dev_read(const vbf_filter* f) {
    if (!f) return nullptr;
    Storage& s = *f->bits;
    std::lock_guard<std::mutex> lk(s.mu);
    if (!hip_forked() && storage_sync(s) != VBF_OK) return nullptr;  // as vbf_filter_words_dev
    return s.d_words;  // read-only use: the mirror and `pristine` stay trusted
}

int vbf_filter_set_num_elements(vbf_filter* f, uint32_t n) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    f->n.store(n);
    return ok();
}

int vbf_filter_set_sst_entries(vbf_filter* f, uint64_t entries) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    f->sst_entries.store(entries);
    return ok();
}
uint64_t vbf_filter_sst_entries(const vbf_filter* f) { return f ? f->sst_entries.load() : VBF_EXT_NONE; }
int vbf_filter_take_restored(vbf_filter* f) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    return f->restored.exchange(0);
}

int vbf_filter_serialize(const vbf_filter* f, uint8_t out[16]) {
    if (!f || !out) return fail(VBF_EINVAL, "NULL argument");
    vbf_meta_serialize(f->k, f->n.load(), f->p, out);
    return ok();
}

int vbf_filter_set_dev(vbf_filter* f, const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
                       uint64_t n, int len_prefix, void* stream) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    std::unique_lock<std::mutex> lk(s.mu);
    int rc = storage_drain(s, lk);
    if (rc) return rc;
    if (s.host()) return host_resident("vbf_filter_set_dev");
    if ((rc = check_mk(s.m, f->k, n))) return rc;
    if ((rc = check_keys(keys, offsets, stride, n))) return rc;
    if (n && f->k) {
        DEVICE_SCOPE(s.device);
        const hipStream_t hs = (hipStream_t)stream;
        if ((rc = storage_wait(s, hs))) return rc;
        vbf::KeyBatch kb = batch(keys, offsets, 0, stride, n, len_prefix);
        s.mirror_ok = false;
        s.pristine = false;
        if ((rc = do_build(kb, s.m, f->k, s.d_words, VBF_BUILD_AUTO, true, hs))) return rc;
        if ((rc = storage_mark(s, hs))) return rc;
        if ((rc = mirror_after_write(s, hs))) return rc;
    }
    f->n.fetch_add((uint32_t)n);
    return ok();
}

int vbf_filter_set_host(vbf_filter* f, const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
                        uint64_t n, int len_prefix) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    int rc = check_mk(s.m, f->k, n);
    if (rc) return rc;
    if ((rc = check_keys(keys, offsets, stride, n))) return rc;
    std::unique_lock<std::mutex> lk(s.mu);
    if ((rc = storage_drain(s, lk))) return rc;
    if (n && f->k) {
        if (s.host()) {
            s.pristine = false;
            host_set(host_words(s), s.m, f->k, keys, offsets, stride, n, len_prefix != 0);
        } else {
            DEVICE_SCOPE(s.device);
            if ((rc = device_set_host(s, f->k, keys, offsets, stride, n, len_prefix))) return rc;
        }
    }
    f->n.fetch_add((uint32_t)n);
    return ok();
}

int vbf_filter_set_host_async(vbf_filter* f, const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
                              uint64_t n, int len_prefix, void (*release)(void*), void* release_ctx) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    int rc = check_mk(s.m, f->k, n);
    if (rc) return rc;
    if ((rc = check_keys(keys, offsets, stride, n))) return rc;
    std::unique_ptr<AsyncJob> j(new AsyncJob());
    j->s = f->bits;
    j->k = f->k;
    j->stride = stride;
    j->n = n;
    j->lp = len_prefix;
    j->release = release;
    j->ctx = release_ctx;
    if (n && f->k && !release) {
        // no release callback: the caller may reuse its buffers on return, so the job runs from
        // the library's own copy
        const uint64_t base = offsets ? offsets[0] : 0;
        const uint64_t bytes = offsets ? offsets[n] - base : n * stride;
        j->own_keys.reset(new (std::nothrow) uint8_t[bytes ? bytes : 1]);
        if (!j->own_keys) return fail(VBF_ENOMEM, "copying %llu key bytes", (unsigned long long)bytes);
        if (bytes) par_memcpy(j->own_keys.get(), keys + base, bytes);
        if (offsets) {
            j->own_offs.reset(new (std::nothrow) uint64_t[n + 1]);
            if (!j->own_offs) return fail(VBF_ENOMEM, "copying %llu offsets", (unsigned long long)(n + 1));
            for (uint64_t i = 0; i <= n; ++i) j->own_offs[i] = offsets[i] - base;
        }
        j->keys = j->own_keys.get();
        j->offsets = j->own_offs.get();
    } else {
        j->keys = keys;
        j->offsets = offsets;
    }
    std::unique_lock<std::mutex> lk(s.mu);
    if (s.host() || !n || !f->k) {  // nothing to overlap with: the CPU set runs now
        if ((rc = storage_drain(s, lk))) return rc;
        if (n && f->k) {
            s.pristine = false;
            host_set(host_words(s), s.m, f->k, j->keys, j->offsets, stride, n, len_prefix != 0);
        }
        lk.unlock();
        if (release) release(release_ctx);
    } else {
        // a forked child: a device-resident filter's set never runs here (HIP is the parent's), so
        // fail before anything is queued or counted -- no job, no worker thread, no n += N
        if (hip_forked()) return fail_forked();
        if (s.jobs_pid != getpid() && s.jobs_done != s.jobs_queued) {
            // forked while the parent had sets queued on this filter: they never run here.  Report
            // that now (as every other call does) instead of overwriting jobs_pid, which would make
            // the parent's jobs look like this process's and every later drain wait forever
            // (ADVICE r04).  The caller keeps its buffers: release is not called on an error.
            (void)storage_jobs_settled(s);
            if ((rc = storage_drain(s, lk))) return rc;
        }
        ++s.jobs_queued;
        s.jobs_pid = getpid();
        s.pristine = false;
        // s.device cannot change while the job is queued: migrate drains first
        AsyncQueue::get(s.device).push(j.release());
    }
    f->n.fetch_add((uint32_t)n);
    return ok();
}

int vbf_filter_sync(vbf_filter* f) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    std::unique_lock<std::mutex> lk(s.mu);
    int rc = storage_drain(s, lk);
    if (rc) return rc;
    if (!s.host()) {
        DEVICE_SCOPE(s.device);
        if ((rc = storage_sync(s))) return rc;
    }
    return ok();
}

int vbf_filter_busy(const vbf_filter* f) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    std::lock_guard<std::mutex> lk(s.mu);
    if (!storage_jobs_settled(s)) return 1;
    if (s.host() || !s.pending) return 0;
    DEVICE_SCOPE(s.device);
    const hipError_t e = hipEventQuery(s.last);
    if (e == hipErrorNotReady) return 1;
    if (e != hipSuccess) return fail(VBF_EHIP, "hipEventQuery: %s", hipGetErrorString(e));
    return 0;
}

int vbf_filter_stream_wait(const vbf_filter* f, void* stream) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    std::unique_lock<std::mutex> lk(s.mu);
    int rc = storage_drain(s, lk);
    if (rc) return rc;
    if (s.host()) return host_resident("vbf_filter_stream_wait");
    DEVICE_SCOPE(s.device);
    if ((rc = storage_wait(s, (hipStream_t)stream))) return rc;
    return ok();
}

int vbf_filter_stream_record(vbf_filter* f, void* stream) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    std::unique_lock<std::mutex> lk(s.mu);
    int rc = storage_drain(s, lk);
    if (rc) return rc;
    if (s.host()) return host_resident("vbf_filter_stream_record");
    DEVICE_SCOPE(s.device);
    s.pristine = false;
    s.ext_write = false;  // the write is declared: the mirror is refreshed behind it from here on
    if ((rc = storage_mark(s, (hipStream_t)stream))) return rc;
    if ((rc = mirror_after_write(s, (hipStream_t)stream))) return rc;
    return ok();
}

int vbf_filter_set_mirror(vbf_filter* f, int mode) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    if (mode < VBF_MIRROR_OFF || mode > VBF_MIRROR_EAGER) return fail(VBF_EINVAL, "unknown mirror mode %d", mode);
    Storage& s = *f->bits;
    std::unique_lock<std::mutex> lk(s.mu);
    int rc = storage_drain(s, lk);
    if (rc) return rc;
    if (!s.host()) {
        DEVICE_SCOPE(s.device);
        if ((rc = storage_sync(s))) return rc;  // a queued eager refresh must land before a free
    }
    s.mirror_mode = mode;
    if (mode == VBF_MIRROR_OFF) s.free_mirror();
    return ok();
}

int vbf_filter_contains_dev(const vbf_filter* f, const uint8_t* keys, const uint64_t* offsets,
                            uint64_t stride, uint64_t n, int len_prefix, uint8_t* out, void* stream) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    std::unique_lock<std::mutex> lk(s.mu);
    int rc = storage_drain(s, lk);
    if (rc) return rc;
    if (s.host()) return host_resident("vbf_filter_contains_dev");
    if ((rc = check_mk(s.m, f->k, n))) return rc;
    if ((rc = check_keys(keys, offsets, stride, n))) return rc;
    if (n && !out) return fail(VBF_EINVAL, "out is NULL");
    if (n == 0) return ok();
    DEVICE_SCOPE(s.device);
    const hipStream_t hs = (hipStream_t)stream;
    if ((rc = storage_wait(s, hs))) return rc;
    vbf::KeyBatch kb = batch(keys, offsets, 0, stride, n, len_prefix);
    if ((rc = do_probe(kb, s.m, f->k, s.d_words, out, nullptr, VBF_BUILD_AUTO, hs))) return rc;
    if ((rc = storage_mark(s, hs))) return rc;  // a later clear / load must not overtake the reads
    return ok();
}

int vbf_filter_contains_host(const vbf_filter* f, const uint8_t* keys, const uint64_t* offsets,
                             uint64_t stride, uint64_t n, int len_prefix, uint8_t* out) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    int rc = check_mk(s.m, f->k, n);
    if (rc) return rc;
    if ((rc = check_keys(keys, offsets, stride, n))) return rc;
    if (n && !out) return fail(VBF_EINVAL, "out is NULL");
    if (n == 0) return ok();
    std::unique_lock<std::mutex> lk(s.mu);
    if ((rc = storage_drain(s, lk))) return rc;
    if (s.host()) {
        host_contains(host_words(s), s.m, f->k, keys, offsets, stride, n, len_prefix != 0, out);
        return ok();
    }
    DEVICE_SCOPE(s.device);
    if (mirror_mode(s) != VBF_MIRROR_OFF && n <= mirror_max_keys()) {
        // the read path's single-key probes (range.rs:130,136,171) answer from the host mirror
        if ((rc = mirror_fill(s))) return rc;
        host_contains(s.mirror, s.m, f->k, keys, offsets, stride, n, len_prefix != 0, out);
        return ok();
    }
    Staging* st = staging_for(s.device);
    std::lock_guard<std::mutex> lk2(st->mu);
    if ((rc = st->init(s.device))) return rc;
    if ((rc = storage_sync(s))) return rc;
    rc = pipeline_host_keys(
        *st, keys, offsets, stride, n, len_prefix, true,
        [&](const vbf::KeyBatch& kb, uint64_t, int b, hipStream_t hs) -> int {
            if (int rc2 = do_probe(kb, s.m, f->k, s.d_words, st->d_out[b], nullptr, VBF_BUILD_AUTO, hs)) return rc2;
            HIP_TRY(hipMemcpyAsync(st->h_out[b], st->d_out[b], kb.n, hipMemcpyDeviceToHost, hs));
            return VBF_OK;
        },
        [&](int b, uint64_t lo, uint64_t cnt) {
            par_memcpy(out + lo, st->h_out[b], cnt);
            return VBF_OK;
        });
    if (rc) return rc;
    return ok();
}

int vbf_filter_clear(vbf_filter* f, vbf_filter** out) {
    if (!f || !out) return fail(VBF_EINVAL, "NULL argument");
    Storage& s = *f->bits;
    int device;
    {
        std::unique_lock<std::mutex> lk(s.mu);
        int rc = storage_drain(s, lk);
        if (rc) return rc;
        if (s.host()) {
            std::fill(s.h_words.begin(), s.h_words.end(), 0u);
        } else {
            DEVICE_SCOPE(s.device);
            hipStream_t fs;
            if ((rc = filter_stream(s.device, &fs))) return rc;
            if ((rc = storage_wait(s, fs))) return rc;  // a pending set_dev must not undo the clear
            if (s.nwords) HIP_TRY(hipMemsetAsync(s.d_words, 0, s.nwords * 4, fs));
            HIP_TRY(hipStreamSynchronize(fs));
            s.pending = false;
            if (s.mirror) {  // the mirror stays exact: all zero too
                std::memset(s.mirror, 0, s.nwords * 4);
                s.mirror_ok = true;
            }
        }
        s.pristine = true;
        device = s.device;
    }
    return make_filter(device, s.m, f->k, f->p, out);
}

// Caller holds s.mu (drained).
static int words_to_host_locked(Storage& s, uint32_t* out) {
    if (!s.nwords) return VBF_OK;
    if (s.host()) {
        if (s.h_words.empty()) std::memset(out, 0, s.nwords * 4);  // never written: all zero
        else std::memcpy(out, s.h_words.data(), s.nwords * 4);
        return VBF_OK;
    }
    DEVICE_SCOPE(s.device);
    int rc = storage_sync(s);  // this filter's pending work only: other filters keep running
    if (rc) return rc;
    if (s.mirror_current()) {  // current host copy: no PCIe transfer
        par_memcpy(out, s.mirror, s.nwords * 4);
        return VBF_OK;
    }
    Staging* st = staging_for(s.device);
    std::lock_guard<std::mutex> lk2(st->mu);
    rc = st->init(s.device);
    if (!rc) rc = xfer_d2h(*st, out, s.d_words, s.nwords * 4);
    return rc;
}

int vbf_filter_words_to_host(const vbf_filter* f, uint32_t* out, uint64_t nwords) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    if (nwords < s.nwords || (s.nwords && !out)) return fail(VBF_EINVAL, "out holds %llu < %llu words",
                                                            (unsigned long long)nwords, (unsigned long long)s.nwords);
    std::unique_lock<std::mutex> lk(s.mu);
    int rc = storage_drain(s, lk);
    if (!rc) rc = words_to_host_locked(s, out);
    return rc ? rc : ok();
}

// Caller holds s.mu (drained).
static int words_from_host_locked(Storage& s, const uint32_t* in) {
    if (!s.nwords) return VBF_OK;
    s.pristine = false;
    if (s.host()) {
        std::memcpy(host_words(s), in, s.nwords * 4);
        return VBF_OK;
    }
    DEVICE_SCOPE(s.device);
    int rc = storage_sync(s);
    if (rc) return rc;
    s.mirror_ok = false;
    Staging* st = staging_for(s.device);
    std::lock_guard<std::mutex> lk2(st->mu);
    rc = st->init(s.device);
    if (!rc) rc = xfer_h2d(*st, s.d_words, in, s.nwords * 4);
    if (!rc && mirror_mode(s) == VBF_MIRROR_EAGER) {
        if (!s.mirror) HIP_TRY(hipHostMalloc((void**)&s.mirror, s.nwords * 4, hipHostMallocDefault));
        par_memcpy(s.mirror, in, s.nwords * 4);
        s.mirror_ok = true;
    }
    return rc;
}

int vbf_filter_words_from_host(vbf_filter* f, const uint32_t* in, uint64_t nwords) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    if (nwords != s.nwords || (s.nwords && !in)) return fail(VBF_EINVAL, "expected %llu words, got %llu",
                                                            (unsigned long long)s.nwords, (unsigned long long)nwords);
    std::unique_lock<std::mutex> lk(s.mu);
    int rc = storage_drain(s, lk);
    if (!rc) rc = words_from_host_locked(s, in);
    return rc ? rc : ok();
}

int vbf_filter_migrate(vbf_filter* f, int device) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    if (device != VBF_DEVICE_HOST) {
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return fail(VBF_ENODEV, "no HIP device available");
        if (device == VBF_DEVICE_AUTO) device = (int)(g_auto_rr.fetch_add(1) % (uint64_t)count);
        if (device < 0 || device >= count) return fail(VBF_ENODEV, "device %d out of range (%d devices)", device, count);
    }
    std::unique_lock<std::mutex> lk(s.mu);
    int rc = storage_drain(s, lk);
    if (rc) return rc;
    if (device == s.device) return ok();
    std::vector<uint32_t> w;
    const bool zeros = s.pristine;  // nothing to copy: the target gets zeroed words
    if (s.host()) {
        w.swap(s.h_words);
        if (!zeros && w.size() != s.nwords) w.assign(s.nwords, 0u);  // written words are allocated
    } else {
        DEVICE_SCOPE(s.device);
        if ((rc = storage_sync(s))) return rc;
        if (!zeros) w.resize(s.nwords);  // to the host, a pristine filter stays unallocated
        if (s.nwords && !zeros) HIP_TRY(hipMemcpy(w.data(), s.d_words, s.nwords * 4, hipMemcpyDeviceToHost));
    }
    uint32_t* nd = nullptr;
    if (device != VBF_DEVICE_HOST && s.nwords) {
        DEVICE_SCOPE(device);
        hipError_t e = hipMalloc((void**)&nd, s.nwords * 4);
        // a pristine filter's words are zeroed asynchronously below (no copy, no host wait)
        if (e == hipSuccess && !zeros) e = hipMemcpy(nd, w.data(), s.nwords * 4, hipMemcpyHostToDevice);
        if (e != hipSuccess) {  // the filter stays where it was, bits intact
            (void)hipGetLastError();
            if (nd) (void)hipFree(nd);
            if (s.host()) s.h_words.swap(w);
            return fail(e == hipErrorOutOfMemory ? VBF_ENOMEM : VBF_EHIP, "moving the bits to device %d: %s",
                        device, hipGetErrorString(e));
        }
    }
    if (!s.host()) {  // release the old device copy (its work is finished: storage_sync above)
        DEVICE_SCOPE(s.device);
        if (s.d_words) (void)hipFree(s.d_words);
        if (s.last) (void)hipEventDestroy(s.last);
        s.last = nullptr;
        s.pending = false;
    }
    // a mirror of the old device copy still holds the bits; moving to the host makes it moot
    if (device == VBF_DEVICE_HOST) s.free_mirror();
    s.d_words = nd;
    if (device == VBF_DEVICE_HOST) s.h_words.swap(w);
    s.device = device;
    if (nd && zeros) {  // on the filter's stream; every later use waits for the filter's last event
        DEVICE_SCOPE(device);
        hipStream_t fs;
        if ((rc = filter_stream(device, &fs))) return rc;
        HIP_TRY(hipMemsetAsync(nd, 0, s.nwords * 4, fs));
        if ((rc = storage_mark(s, fs))) return rc;
    }
    return ok();
}

// ---- persisted bit array ----

static constexpr uint32_t kExtMagic = 0x57464256u;  // "VBFW"
static constexpr uint32_t kExtVersion = 2;
static constexpr uint64_t kExtBytes = 32;  // u32 magic | u32 version | u32 m | u32 nwords | u64 entries | u64 checksum

static inline void put_u32(uint8_t* p, uint32_t v) { std::memcpy(p, &v, 4); }
static inline void put_u64(uint8_t* p, uint64_t v) { std::memcpy(p, &v, 8); }
static inline uint32_t get_u32(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}
static inline uint64_t get_u64(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
}

int vbf_filter_serialize_ext(const vbf_filter* f, const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
                             uint64_t entries, int len_prefix, uint8_t* buf, uint64_t cap, uint64_t* len) {
    if (!f || !len) return fail(VBF_EINVAL, "NULL argument");
    Storage& s = *f->bits;
    const uint32_t k = f->k, n = f->n.load();
    const double p = f->p;
    // recover_meta (bf.rs:144-147) recreates m from the stored n; persisted bits are useful only
    // in that shape
    const uint32_t m_rec = vbf_num_bits((uint64_t)n, p);
    const uint64_t nw = ((uint64_t)m_rec + 31) / 32;
    enum { kHeaderOnly, kOwnWords, kFromKeys } mode = kHeaderOnly;
    if (entries != VBF_EXT_NONE && !(m_rec == 0 && k > 0 && entries > 0)) {
        if (s.m == m_rec) mode = kOwnWords;
        else if (keys || offsets || entries == 0) mode = kFromKeys;
    }
    if (mode == kFromKeys) {
        int rc = check_keys(keys, offsets, stride, entries);
        if (rc) return rc;
    }
    const uint64_t need = 16 + (mode == kHeaderOnly ? 0 : kExtBytes + nw * 4);
    *len = need;
    if (!buf) return ok();  // size query
    if (cap < need) return fail(VBF_EINVAL, "buffer holds %llu < %llu bytes", (unsigned long long)cap,
                                (unsigned long long)need);
    vbf_meta_serialize(k, n, p, buf);
    if (mode == kHeaderOnly) return ok();
    uint8_t* body = buf + 16 + kExtBytes;
    const bool aligned = ((uintptr_t)body & 3) == 0;
    std::vector<uint32_t> tmp;
    uint32_t* w = reinterpret_cast<uint32_t*>(body);
    if (!aligned) {
        tmp.resize(nw);
        w = tmp.data();
    }
    int rc = VBF_OK;
    if (mode == kOwnWords) {
        std::unique_lock<std::mutex> lk(s.mu);
        rc = storage_drain(s, lk);
        if (!rc) rc = words_to_host_locked(s, w);
    } else {
        std::memset(w, 0, nw * 4);
        if (entries && k) {
            int device;
            {
                std::lock_guard<std::mutex> lk(s.mu);
                device = s.device;
            }
            if (device == VBF_DEVICE_HOST) host_set(w, m_rec, k, keys, offsets, stride, entries, len_prefix != 0);
            else rc = vbf_build_host(keys, offsets, stride, entries, len_prefix, m_rec, k, w, nw, device);
        }
    }
    if (rc) return rc;
    if (!aligned) std::memcpy(body, tmp.data(), nw * 4);
    uint8_t* e = buf + 16;
    put_u32(e, kExtMagic);
    put_u32(e + 4, kExtVersion);
    put_u32(e + 8, m_rec);
    put_u32(e + 12, (uint32_t)nw);
    put_u64(e + 16, entries);
    put_u64(e + 24, words_checksum(w, nw));
    return ok();
}

int vbf_filter_recover_ext(const uint8_t* bytes, uint64_t len, int device, vbf_filter** out, int* restored) {
    if (!bytes || !out) return fail(VBF_EINVAL, "NULL argument");
    if (restored) *restored = 0;
    vbf_filter* f = nullptr;
    int rc = vbf_filter_recover(bytes, (size_t)len, device, &f);
    if (rc) return rc;
    const uint32_t m = f->bits->m;
    const uint64_t nw = ((uint64_t)m + 31) / 32;
    if (len >= 16 + kExtBytes) {
        const uint8_t* e = bytes + 16;
        const uint8_t* body = e + kExtBytes;
        if (get_u32(e) == kExtMagic && get_u32(e + 4) == kExtVersion && get_u32(e + 8) == m &&
            get_u32(e + 12) == nw && len - 16 - kExtBytes == nw * 4) {
            std::vector<uint32_t> tmp;
            const uint32_t* w = reinterpret_cast<const uint32_t*>(body);
            if ((uintptr_t)body & 3) {
                tmp.resize(nw);
                std::memcpy(tmp.data(), body, nw * 4);
                w = tmp.data();
            }
            if (words_checksum(w, nw) == get_u64(e + 24)) {
                if ((rc = vbf_filter_words_from_host(f, w, nw))) {
                    vbf_filter_free(f);
                    return rc;
                }
                // recover_meta + build_filter_from_entries (range.rs:121-124): stored n + entries
                f->n.store((uint32_t)(f->n.load() + get_u64(e + 16)));
                f->restored.store(1);
                if (restored) *restored = 1;
            }
        }
    }
    *out = f;
    return ok();
}

// ---- SST data.db decode ----

int vbf_sst_index_blocks(const uint8_t* index, uint64_t len, uint32_t* offsets, uint64_t cap, uint64_t* nblocks) {
    if (!nblocks || (len && !index)) return fail(VBF_EINVAL, "NULL argument");
    std::vector<uint32_t> v;
    int rc = parse_index(index, len, &v);
    if (rc) return rc;
    *nblocks = v.size();
    if (offsets && cap) memcpy(offsets, v.data(), 4 * std::min<uint64_t>(cap, v.size()));
    return ok();
}

int vbf_sst_decode_dev(const uint8_t* data, uint64_t len, const uint32_t* blocks, uint64_t nblocks, uint8_t* keys,
                       uint64_t keys_cap, uint64_t* offsets, uint32_t* val_offsets, uint64_t* created_ms,
                       uint8_t* tombstones, uint64_t entries_cap, uint64_t* n_out, void* stream) {
    FORK_GUARD();
    if (!n_out) return fail(VBF_EINVAL, "n_out is NULL");
    hipStream_t s = (hipStream_t)stream;
    vbf::SstArgs a;
    int rc = sst_count_pass(data, len, blocks, nblocks, s, &a, n_out);
    if (rc) return rc;
    const uint64_t n = *n_out, kb = len - 17 * n;
    if ((val_offsets || created_ms || tombstones) && entries_cap < n)
        return fail(VBF_EINVAL, "entry arrays hold %llu < %llu entries", (unsigned long long)entries_cap,
                    (unsigned long long)n);
    if (offsets && entries_cap < n + 1)
        return fail(VBF_EINVAL, "offsets holds %llu < %llu entries", (unsigned long long)entries_cap,
                    (unsigned long long)(n + 1));
    if (keys && keys_cap < kb)
        return fail(VBF_EINVAL, "keys holds %llu < %llu bytes", (unsigned long long)keys_cap, (unsigned long long)kb);
    if ((rc = sst_emit_pass(a, keys, offsets, val_offsets, created_ms, tombstones, s))) return rc;
    return ok();
}

int vbf_sst_decode_host(const uint8_t* data, uint64_t len, const uint8_t* index, uint64_t index_len, uint8_t* keys,
                        uint64_t keys_cap, uint64_t* offsets, uint32_t* val_offsets, uint64_t* created_ms,
                        uint8_t* tombstones, uint64_t entries_cap, uint64_t* n_out, int device) {
    if (!n_out || (len && !data) || (index_len && !index)) return fail(VBF_EINVAL, "NULL argument");
    std::vector<uint32_t> blk;
    int rc = parse_index(index, index_len, &blk);
    if (rc) return rc;
    DEVICE_SCOPE(device);
    hipStream_t s;
    if ((rc = filter_stream(device, &s))) return rc;
    // device image: data | blocks | then the outputs (count pass first, to size them)
    const uint64_t o_blk = align256(len), o_end = o_blk + align256(blk.size() * 4);
    void* in = nullptr;
    if ((rc = get_workspace(s, o_end, &in, kWsSstInput))) return rc;
    uint8_t* d_data = static_cast<uint8_t*>(in);
    uint32_t* d_blk = reinterpret_cast<uint32_t*>(d_data + o_blk);
    if (len) HIP_TRY(hipMemcpyAsync(d_data, data, len, hipMemcpyHostToDevice, s));
    if (blk.size()) HIP_TRY(hipMemcpyAsync(d_blk, blk.data(), blk.size() * 4, hipMemcpyHostToDevice, s));
    vbf::SstArgs a;
    if ((rc = sst_count_pass(d_data, len, d_blk, blk.size(), s, &a, n_out))) return rc;
    const uint64_t n = *n_out, kb = len - 17 * n;
    if ((val_offsets || created_ms || tombstones) && entries_cap < n)
        return fail(VBF_EINVAL, "entry arrays hold %llu < %llu entries", (unsigned long long)entries_cap,
                    (unsigned long long)n);
    if (offsets && entries_cap < n + 1)
        return fail(VBF_EINVAL, "offsets holds %llu < %llu entries", (unsigned long long)entries_cap,
                    (unsigned long long)(n + 1));
    if (keys && keys_cap < kb)
        return fail(VBF_EINVAL, "keys holds %llu < %llu bytes", (unsigned long long)keys_cap, (unsigned long long)kb);
    const uint64_t o_keys = 0, o_off = align256(kb), o_val = o_off + align256((n + 1) * 8);
    const uint64_t o_cr = o_val + align256(n * 4), o_tb = o_cr + align256(n * 8), total = o_tb + align256(n);
    void* out = nullptr;
    if ((rc = get_workspace(s, total, &out, kWsSstKeys))) return rc;
    char* ob = static_cast<char*>(out);
    uint8_t* d_keys = keys ? reinterpret_cast<uint8_t*>(ob + o_keys) : nullptr;
    uint64_t* d_off = offsets ? reinterpret_cast<uint64_t*>(ob + o_off) : nullptr;
    uint32_t* d_val = val_offsets ? reinterpret_cast<uint32_t*>(ob + o_val) : nullptr;
    uint64_t* d_cr = created_ms ? reinterpret_cast<uint64_t*>(ob + o_cr) : nullptr;
    uint8_t* d_tb = tombstones ? reinterpret_cast<uint8_t*>(ob + o_tb) : nullptr;
    if ((rc = sst_emit_pass(a, d_keys, d_off, d_val, d_cr, d_tb, s))) return rc;
    if (keys && kb) HIP_TRY(hipMemcpyAsync(keys, d_keys, kb, hipMemcpyDeviceToHost, s));
    if (offsets) HIP_TRY(hipMemcpyAsync(offsets, d_off, (n + 1) * 8, hipMemcpyDeviceToHost, s));
    if (val_offsets && n) HIP_TRY(hipMemcpyAsync(val_offsets, d_val, n * 4, hipMemcpyDeviceToHost, s));
    if (created_ms && n) HIP_TRY(hipMemcpyAsync(created_ms, d_cr, n * 8, hipMemcpyDeviceToHost, s));
    if (tombstones && n) HIP_TRY(hipMemcpyAsync(tombstones, d_tb, n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return ok();
}

// range.rs:117-128 (load_entries_from_file + build_filter_from_entries) on the device: decode
// data.db into packed keys/offsets and OR their bits into the filter; no_of_elements += n.
// Caller holds s.mu (drained), on s.device; the filter is device-resident.
static int rebuild_locked(vbf_filter* f, Storage& s, const uint8_t* data, uint64_t len, const uint32_t* blocks,
                          uint64_t nblocks, uint64_t* n_out, hipStream_t st) {
    uint64_t n = 0;
    vbf::SstArgs a;
    uint32_t ulen = 0xFFFFFFFFu;
    int rc = sst_count_pass(data, len, blocks, nblocks, st, &a, &n, &ulen);
    if (rc) return rc;
    if (n_out) *n_out = n;
    if ((rc = check_mk(s.m, f->k, n))) return rc;
    if (n && f->k) {
        const uint64_t kb = len - 17 * n, o_off = align256(kb);
        void* out = nullptr;
        if ((rc = get_workspace(st, o_off + (n + 1) * 8, &out, kWsSstKeys))) return rc;
        uint8_t* d_keys = static_cast<uint8_t*>(out);
        uint64_t* d_off = reinterpret_cast<uint64_t*>(d_keys + o_off);
        // every key the same length (the common case): packed keys are a fixed-stride batch, which
        // the build reads with its aligned fast path instead of through offsets
        const bool uniform = ulen != 0xFFFFFFFFu && ulen > 0;
        if ((rc = sst_emit_pass(a, d_keys, uniform ? nullptr : d_off, nullptr, nullptr, nullptr, st))) return rc;
        if ((rc = storage_wait(s, st))) return rc;
        vbf::KeyBatch kb2 = uniform ? batch(d_keys, nullptr, 0, ulen, n, 1) : batch(d_keys, d_off, 0, 0, n, 1);
        s.mirror_ok = false;
        s.pristine = false;
        if ((rc = do_build(kb2, s.m, f->k, s.d_words, VBF_BUILD_AUTO, true, st))) return rc;
        if ((rc = storage_mark(s, st))) return rc;
        if ((rc = mirror_after_write(s, st))) return rc;
    }
    f->n.fetch_add((uint32_t)n);
    return VBF_OK;
}

int vbf_filter_rebuild_from_sst_dev(vbf_filter* f, const uint8_t* data, uint64_t len, const uint32_t* blocks,
                                    uint64_t nblocks, uint64_t* n_out, void* stream) {
    if (!f) return fail(VBF_EINVAL, "filter is NULL");
    Storage& s = *f->bits;
    std::unique_lock<std::mutex> lk(s.mu);
    int rc = storage_drain(s, lk);
    if (rc) return rc;
    if (s.host()) return host_resident("vbf_filter_rebuild_from_sst_dev");
    DEVICE_SCOPE(s.device);
    if ((rc = rebuild_locked(f, s, data, len, blocks, nblocks, n_out, (hipStream_t)stream))) return rc;
    return ok();
}

int vbf_filter_rebuild_from_sst_host(vbf_filter* f, const uint8_t* data, uint64_t len, const uint8_t* index,
                                     uint64_t index_len, uint64_t* n_out) {
    if (!f || (len && !data) || (index_len && !index)) return fail(VBF_EINVAL, "NULL argument");
    Storage& s = *f->bits;
    std::vector<uint32_t> blk;
    int rc = parse_index(index, index_len, &blk);
    if (rc) return rc;
    std::unique_lock<std::mutex> lk(s.mu);
    if ((rc = storage_drain(s, lk))) return rc;
    if (s.host()) return host_resident("vbf_filter_rebuild_from_sst_host");
    DEVICE_SCOPE(s.device);
    hipStream_t st;
    if ((rc = filter_stream(s.device, &st))) return rc;
    const uint64_t o_blk = align256(len), o_end = o_blk + align256(blk.size() * 4);
    void* in = nullptr;
    if ((rc = get_workspace(st, o_end, &in, kWsSstInput))) return rc;
    uint8_t* d_data = static_cast<uint8_t*>(in);
    uint32_t* d_blk = reinterpret_cast<uint32_t*>(d_data + o_blk);
    if (len) HIP_TRY(hipMemcpyAsync(d_data, data, len, hipMemcpyHostToDevice, st));
    if (blk.size()) HIP_TRY(hipMemcpyAsync(d_blk, blk.data(), blk.size() * 4, hipMemcpyHostToDevice, st));
    if ((rc = rebuild_locked(f, s, d_data, len, d_blk, blk.size(), n_out, st))) return rc;
    HIP_TRY(hipStreamSynchronize(st));
    return ok();
}

}  // extern "C"

// ---- batched probe across SSTs ----

namespace {
// Locks every distinct storage of `filters` in address order (clones share one), so two
// concurrent multi-probes over overlapping sets cannot deadlock; then drains each filter's
// queued asynchronous sets.
struct MultiLock {
    std::vector<std::unique_lock<std::mutex>> locks;
    std::vector<Storage*> v;
    explicit MultiLock(const vbf_filter* const* filters, uint32_t nsst) {
        for (uint32_t s = 0; s < nsst; ++s)
            if (filters[s]) v.push_back(filters[s]->bits.get());
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        for (Storage* st : v) locks.emplace_back(st->mu);
    }
    // A device's worker runs its queued jobs in order, each under its own filter's lock.  Waiting
    // for filter A's job while holding B's lock would deadlock when B's job is queued ahead of
    // A's on the same worker.  So: with every lock held, find a filter whose jobs are
    // not all done; if there is one, release every lock, wait for that filter alone, take the
    // locks again (address order) and look again.  Only once all are settled are failures
    // reported (storage_drain no longer waits then).
    int drain() {
        for (;;) {
            Storage* behind = nullptr;
            for (Storage* st : v)
                if (!storage_jobs_settled(*st)) {
                    behind = st;
                    break;
                }
            if (!behind) break;
            for (auto& l : locks) l.unlock();
            {
                std::unique_lock<std::mutex> lk(behind->mu);
                behind->jobs_cv.wait(lk, [&] { return storage_jobs_settled(*behind); });
            }
            for (auto& l : locks) l.lock();
        }
        for (size_t i = 0; i < v.size(); ++i)
            if (int rc = storage_drain(*v[i], locks[i])) return rc;
        return VBF_OK;
    }
};

// Rust's Ord for [u8]: bytewise, then shorter first.
int cmp_host(const uint8_t* a, uint64_t la, const uint8_t* b, uint64_t lb) {
    const int c = std::memcmp(a, b, std::min(la, lb));
    if (c) return c < 0 ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// The read path's small batches (one get: one key against every in-range SST,
// range.rs:101-136) answered on the CPU from the filters' host mirrors; the same answers as the
// k_multi_probe kernel.  Caller holds every filter's lock (drained).  The filters may live on
// different GPUs (compaction places them round-robin, VBF_DEVICE_AUTO): each mirror is filled on
// its own device.
static int mirror_fill_on_device(Storage& s) {
    DEVICE_SCOPE(s.device);
    return mirror_fill(s);
}

int multi_probe_mirror(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n, int len_prefix,
                       uint32_t nsst, const vbf_filter* const* filters, const uint8_t* bounds,
                       const uint64_t* bounds_off, uint8_t* out) {
    for (uint32_t i = 0; i < nsst; ++i)
        if (int rc = mirror_fill_on_device(*filters[i]->bits)) return rc;
    for (uint64_t j = 0; j < n; ++j) {
        const uint8_t* kp;
        uint64_t kl;
        host_key(keys, offsets, stride, j, &kp, &kl);
        for (uint32_t i = 0; i < nsst; ++i) {
            const Storage& st = *filters[i]->bits;
            const uint32_t k = filters[i]->k;
            bool hit = true;
            if (bounds_off)  // range.rs:118
                hit = cmp_host(kp, kl, bounds + bounds_off[2 * i], bounds_off[2 * i + 1] - bounds_off[2 * i]) >= 0 &&
                      cmp_host(kp, kl, bounds + bounds_off[2 * i + 1], bounds_off[2 * i + 2] - bounds_off[2 * i + 1]) <= 0;
            if (hit && k > 0 && st.m == 0)
                return fail(VBF_EDIVZERO, "a key inside an SST's range reaches its filter with m == 0 < k "
                                          "(bf.rs:100 divides by zero)");
            uint8_t h = hit ? 1 : 0;
            if (hit && k > 0) host_contains(st.mirror, st.m, k, kp, nullptr, kl, 1, len_prefix != 0, &h);
            out[j * nsst + i] = h;
        }
    }
    return VBF_OK;
}

int multi_probe(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n, int len_prefix,
                uint32_t nsst, const vbf_filter* const* filters, const uint8_t* bounds, const uint64_t* bounds_off,
                uint8_t* out, hipStream_t s) {
    if (nsst && !filters) return fail(VBF_EINVAL, "filters is NULL");
    bool zero_m = false;
    for (uint32_t i = 0; i < nsst; ++i) {
        if (!filters[i]) return fail(VBF_EINVAL, "filters[%u] is NULL", i);
        if (filters[i]->bits->host()) return host_resident("vbf_multi_probe");
        if (filters[i]->bits->device != filters[0]->bits->device)
            return fail(VBF_EINVAL, "filters[%u] lives on device %d, filters[0] on %d", i, filters[i]->bits->device,
                        filters[0]->bits->device);
        // bf.rs:100 divides by m: the reference panics once a key reaches such a filter.  Without
        // key ranges every key reaches every filter; with them only keys inside its range do.
        if (filters[i]->bits->m == 0 && filters[i]->k > 0 && n) {
            if (!bounds_off)
                return fail(VBF_EDIVZERO, "filters[%u]: m == 0 with k = %u (bf.rs:100 divides by zero)", i,
                            filters[i]->k);
            zero_m = true;
        }
    }
    if (bounds_off) {
        for (uint32_t i = 0; i < 2 * nsst; ++i)
            if (bounds_off[i + 1] < bounds_off[i]) return fail(VBF_EINVAL, "bounds_off not nondecreasing at %u", i);
        if (bounds_off[2 * nsst] && !bounds) return fail(VBF_EINVAL, "bounds is NULL");
    }
    if (!n || !nsst) return VBF_OK;
    if (!out) return fail(VBF_EINVAL, "out is NULL");
    // Filters sharing (m, k) test the same positions for a key: interleave up to 8 of them and
    // probe them together (vbf_multi_part.hip) when the batch is large; the rest one lane per key.
    const char* menv = getenv("VBF_MULTI");  // A/B knob, read per call
    const int mode = menv ? atoi(menv) : 0;
    std::vector<vbf::MultiGroup> groups;
    std::vector<char> grouped(nsst, 0);
    if (mode != 1 && (mode == 2 || n >= kMultiGroupMinKeys)) {
        std::vector<uint32_t> order(nsst);
        for (uint32_t i = 0; i < nsst; ++i) order[i] = i;
        auto key_of = [&](uint32_t i) { return std::make_pair(filters[i]->bits->m, filters[i]->k); };
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return key_of(a) < key_of(b); });
        for (uint32_t x = 0; x < nsst;) {
            uint32_t y = x;
            while (y < nsst && key_of(order[y]) == key_of(order[x])) ++y;
            const uint32_t m = filters[order[x]]->bits->m, k = filters[order[x]]->k;
            if (y - x >= 2 && vbf::multi_group_supported(m, k)) {
                for (uint32_t a = x; a < y; a += vbf::kMaxGroup) {
                    vbf::MultiGroup g{};
                    g.m = m;
                    g.k = k;
                    g.G = std::min<uint32_t>(vbf::kMaxGroup, y - a);
                    for (uint32_t q = 0; q < g.G; ++q) {
                        const uint32_t i = order[a + q];
                        g.words[q] = filters[i]->bits->d_words;
                        g.col[q] = i;
                        if (bounds_off) {
                            g.lo_beg[q] = bounds_off[2 * i];
                            g.lo_end[q] = g.hi_beg[q] = bounds_off[2 * i + 1];
                            g.hi_end[q] = bounds_off[2 * i + 2];
                        }
                        grouped[i] = 1;
                    }
                    groups.push_back(g);
                }
            }
            x = y;
        }
    }
    std::vector<vbf::MultiSst> tab;
    for (uint32_t i = 0; i < nsst; ++i) {
        if (grouped[i]) continue;
        const Storage& st = *filters[i]->bits;
        vbf::MultiSst e{st.d_words, st.m, st.m ? ~0ull / st.m : 0, filters[i]->k, i, 0, 0, 0, 0};
        if (bounds_off) {
            e.lo_beg = bounds_off[2 * i];
            e.lo_end = e.hi_beg = bounds_off[2 * i + 1];
            e.hi_end = bounds_off[2 * i + 2];
        }
        tab.push_back(e);
    }
    const uint64_t nb = bounds_off ? bounds_off[2 * nsst] : 0;
    const uint64_t o_b = align256(nsst * sizeof(vbf::MultiSst));
    const uint64_t o_err = o_b + align256(nb + 8);
    void* ws = nullptr;
    int rc = get_workspace(s, o_err + 256, &ws, kWsMulti);
    if (rc) return rc;
    uint32_t* d_err = reinterpret_cast<uint32_t*>(static_cast<char*>(ws) + o_err);
    // the table is read by this launch only; the stream orders reuse by the next call
    if (!tab.empty())
        HIP_TRY(hipMemcpyAsync(ws, tab.data(), tab.size() * sizeof(vbf::MultiSst), hipMemcpyHostToDevice, s));
    uint8_t* d_bounds = nullptr;
    if (bounds_off) {
        d_bounds = static_cast<uint8_t*>(ws) + o_b;
        if (nb) HIP_TRY(hipMemcpyAsync(d_bounds, bounds, nb, hipMemcpyHostToDevice, s));
    }
    if (zero_m) HIP_TRY(hipMemsetAsync(d_err, 0, 4, s));
    HIP_TRY(hipStreamSynchronize(s));  // pageable sources: keep them alive only for this call
    // every filter's pending work (set_dev on another stream) lands before the probe reads it
    for (uint32_t i = 0; i < nsst; ++i)
        if ((rc = storage_wait(*filters[i]->bits, s))) return rc;
    const vbf::KeyBatch kb = batch(keys, offsets, 0, stride, n, len_prefix);
    for (const vbf::MultiGroup& g : groups) {
        const uint64_t need = vbf::multi_group_workspace_bytes(n, g.m, g.k);
        void* gw = nullptr;
        if ((rc = get_workspace(s, need, &gw, kWsMultiGroup))) return rc;
        HIP_TRY(vbf::launch_multi_probe_group(kb, g, d_bounds, out, nsst, gw, need, s));
    }
    if (!tab.empty()) {
        vbf::MultiArgs a{keys, offsets, 0, stride, n, (uint32_t)tab.size(),
                         static_cast<const vbf::MultiSst*>(ws), d_bounds, out, d_err, nsst};
        HIP_TRY(vbf::launch_multi_probe(a, len_prefix != 0, s));
    }
    for (uint32_t i = 0; i < nsst; ++i)
        if ((rc = storage_mark(*filters[i]->bits, s))) return rc;
    if (zero_m) {  // rare (Default / p > 1 filters): one readback decides whether the reference panics
        uint32_t e = 0;
        HIP_TRY(hipMemcpyAsync(&e, d_err, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (e) return fail(VBF_EDIVZERO, "a key inside an SST's range reaches its filter with m == 0 < k "
                                         "(bf.rs:100 divides by zero)");
    }
    return VBF_OK;
}
}  // namespace

extern "C" {

int vbf_multi_probe_dev(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n, int len_prefix,
                        uint32_t nsst, const vbf_filter* const* filters, const uint8_t* bounds,
                        const uint64_t* bounds_off, uint8_t* out, void* stream) {
    FORK_GUARD();
    int rc = check_keys(keys, offsets, stride, n);
    if (rc) return rc;
    if (nsst && filters && filters[0]) {
        MultiLock lk(filters, nsst);
        if ((rc = lk.drain())) return rc;
        if (filters[0]->bits->host()) return host_resident("vbf_multi_probe_dev");
        DEVICE_SCOPE(filters[0]->bits->device);
        if ((rc = multi_probe(keys, offsets, stride, n, len_prefix, nsst, filters, bounds, bounds_off, out,
                              (hipStream_t)stream)))
            return rc;
        return ok();
    }
    if ((rc = multi_probe(keys, offsets, stride, n, len_prefix, nsst, filters, bounds, bounds_off, out,
                          (hipStream_t)stream)))
        return rc;
    return ok();
}

}  // extern "C"

namespace {
// The device path of vbf_multi_probe_host for filters that all live on `device`: the keys are
// staged to it and the answers copied back.  Caller holds every filter's lock (drained).
int multi_probe_host_device(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                            int len_prefix, uint32_t nsst, const vbf_filter* const* filters, const uint8_t* bounds,
                            const uint64_t* bounds_off, uint8_t* out, int device) {
    DEVICE_SCOPE(device);
    hipStream_t s;
    int rc = filter_stream(device, &s);
    if (rc) return rc;
    const uint64_t kbytes = offsets ? offsets[n] - offsets[0] : n * stride;
    const uint64_t o_off = align256(kbytes), o_out = o_off + align256(offsets ? (n + 1) * 8 : 0);
    void* ws = nullptr;
    if ((rc = get_workspace(s, o_out + n * nsst, &ws, kWsMultiKeys))) return rc;
    uint8_t* d_keys = static_cast<uint8_t*>(ws);
    uint64_t* d_off = offsets ? reinterpret_cast<uint64_t*>(d_keys + o_off) : nullptr;
    uint8_t* d_out = d_keys + o_out;
    if (kbytes) HIP_TRY(hipMemcpyAsync(d_keys, keys + (offsets ? offsets[0] : 0), kbytes, hipMemcpyHostToDevice, s));
    if (offsets) {
        // rebase to absolute positions in the device copy
        std::vector<uint64_t> o(offsets, offsets + n + 1);
        const uint64_t b0 = o[0];
        for (auto& x : o) x -= b0;
        HIP_TRY(hipMemcpyAsync(d_off, o.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    if ((rc = multi_probe(d_keys, d_off, stride, n, len_prefix, nsst, filters, bounds, bounds_off, d_out, s)))
        return rc;
    HIP_TRY(hipMemcpyAsync(out, d_out, n * nsst, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return VBF_OK;
}

// vbf_multi_probe_host over filters split into groups (group[i] of filter i; the multi-device
// path groups by device): each group is probed on the device of its first filter, with the keys
// staged there, its filters' bound bytes re-based into a bounds array of their own, and its answer
// columns scattered back into out[n][nsst].  Caller holds every filter's lock (drained).
int multi_probe_host_groups(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                            int len_prefix, uint32_t nsst, const vbf_filter* const* filters, const uint8_t* bounds,
                            const uint64_t* bounds_off, uint8_t* out, const int* group) {
    std::vector<int> gs;
    for (uint32_t i = 0; i < nsst; ++i)
        if (std::find(gs.begin(), gs.end(), group[i]) == gs.end()) gs.push_back(group[i]);
    std::vector<const vbf_filter*> sub;
    std::vector<uint32_t> cols;
    std::vector<uint8_t> sb, tmp;
    std::vector<uint64_t> so;
    for (const int g : gs) {
        sub.clear();
        cols.clear();
        sb.clear();
        so.assign(1, 0);
        for (uint32_t i = 0; i < nsst; ++i) {
            if (group[i] != g) continue;
            sub.push_back(filters[i]);
            cols.push_back(i);
            if (bounds_off) {  // this filter's [lo, hi) bound bytes, re-based
                sb.insert(sb.end(), bounds + bounds_off[2 * i], bounds + bounds_off[2 * i + 1]);
                so.push_back(sb.size());
                sb.insert(sb.end(), bounds + bounds_off[2 * i + 1], bounds + bounds_off[2 * i + 2]);
                so.push_back(sb.size());
            }
        }
        const uint32_t ns = (uint32_t)sub.size();
        const int dev = sub[0]->bits->device;
        for (const vbf_filter* f : sub)
            if (f->bits->device != dev)
                return fail(VBF_EINVAL, "a group's filters live on devices %d and %d", dev, f->bits->device);
        tmp.resize(n * ns);
        if (int rc = multi_probe_host_device(keys, offsets, stride, n, len_prefix, ns, sub.data(),
                                             bounds_off ? sb.data() : nullptr, bounds_off ? so.data() : nullptr,
                                             tmp.data(), dev))
            return rc;
        for (uint64_t j = 0; j < n; ++j)
            for (uint32_t q = 0; q < ns; ++q) out[j * nsst + cols[q]] = tmp[j * ns + q];
    }
    return VBF_OK;
}
}  // namespace

extern "C" {

int vbf_multi_probe_host(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n, int len_prefix,
                         uint32_t nsst, const vbf_filter* const* filters, const uint8_t* bounds,
                         const uint64_t* bounds_off, uint8_t* out) {
    int rc = check_keys(keys, offsets, stride, n);
    if (rc) return rc;
    if (!nsst || !n) {
        if ((rc = multi_probe(keys, offsets, stride, n, len_prefix, nsst, filters, bounds, bounds_off, out, nullptr)))
            return rc;
        return ok();
    }
    if (!filters) return fail(VBF_EINVAL, "filters is NULL");
    for (uint32_t i = 0; i < nsst; ++i)
        if (!filters[i]) return fail(VBF_EINVAL, "filters[%u] is NULL", i);
    if (!out) return fail(VBF_EINVAL, "out is NULL");
    if (bounds_off) {
        for (uint32_t i = 0; i < 2 * nsst; ++i)
            if (bounds_off[i + 1] < bounds_off[i]) return fail(VBF_EINVAL, "bounds_off not nondecreasing at %u", i);
        if (bounds_off[2 * nsst] && !bounds) return fail(VBF_EINVAL, "bounds is NULL");
    }
    MultiLock lk(filters, nsst);
    if ((rc = lk.drain())) return rc;
    bool mirrored = n <= mirror_max_keys();
    std::vector<int> devices;
    for (uint32_t i = 0; i < nsst; ++i) {
        const Storage& st = *filters[i]->bits;
        if (st.host()) return host_resident("vbf_multi_probe_host");
        if (mirror_mode(st) == VBF_MIRROR_OFF) mirrored = false;
        if (std::find(devices.begin(), devices.end(), st.device) == devices.end()) devices.push_back(st.device);
    }
    if (mirrored) {  // the read path's one-key gets: no kernel, any mix of devices
        if ((rc = multi_probe_mirror(keys, offsets, stride, n, len_prefix, nsst, filters, bounds, bounds_off, out)))
            return rc;
        return ok();
    }
    if (devices.size() == 1) {
        if ((rc = multi_probe_host_device(keys, offsets, stride, n, len_prefix, nsst, filters, bounds, bounds_off, out,
                                          devices[0])))
            return rc;
        return ok();
    }
    // filters on several GPUs: each device probes its own filters
    std::vector<int> group(nsst);
    for (uint32_t i = 0; i < nsst; ++i) group[i] = filters[i]->bits->device;
    if ((rc = multi_probe_host_groups(keys, offsets, stride, n, len_prefix, nsst, filters, bounds, bounds_off, out,
                                      group.data())))
        return rc;
    return ok();
}

int vbf_multi_probe_host_grouped(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                                 int len_prefix, uint32_t nsst, const vbf_filter* const* filters,
                                 const uint8_t* bounds, const uint64_t* bounds_off, const int* group, uint8_t* out) {
    int rc = check_keys(keys, offsets, stride, n);
    if (rc) return rc;
    if (!nsst || !n) return ok();
    if (!filters || !group || !out) return fail(VBF_EINVAL, "NULL argument");
    for (uint32_t i = 0; i < nsst; ++i)
        if (!filters[i]) return fail(VBF_EINVAL, "filters[%u] is NULL", i);
    if (bounds_off) {
        for (uint32_t i = 0; i < 2 * nsst; ++i)
            if (bounds_off[i + 1] < bounds_off[i]) return fail(VBF_EINVAL, "bounds_off not nondecreasing at %u", i);
        if (bounds_off[2 * nsst] && !bounds) return fail(VBF_EINVAL, "bounds is NULL");
    }
    MultiLock lk(filters, nsst);
    if ((rc = lk.drain())) return rc;
    for (uint32_t i = 0; i < nsst; ++i)
        if (filters[i]->bits->host()) return host_resident("vbf_multi_probe_host_grouped");
    if ((rc = multi_probe_host_groups(keys, offsets, stride, n, len_prefix, nsst, filters, bounds, bounds_off, out,
                                      group)))
        return rc;
    return ok();
}

}  // extern "C"

// ---- compaction merge ----

namespace {
int compact_merge(const uint8_t* keys, const uint64_t* offsets, const int64_t* created, const uint8_t* tomb,
                  const uint64_t* run_off, uint32_t nruns, const uint8_t* map_keys, const uint64_t* map_off,
                  const int64_t* map_time, uint64_t map_n, int use_ttl, uint64_t entry_ttl_ms, uint64_t tomb_ttl_ms,
                  uint64_t now_ms, uint32_t* out_ids, uint64_t* n_out, uint32_t* upd_ids, int64_t* upd_time,
                  uint64_t* n_upd, hipStream_t s) {
    if (!n_out) return fail(VBF_EINVAL, "n_out is NULL");
    *n_out = 0;
    if (n_upd) *n_upd = 0;
    if (nruns == 0) return VBF_OK;
    if (!run_off || run_off[0] != 0) return fail(VBF_EINVAL, "run_off must start at 0");
    for (uint32_t r = 0; r < nruns; ++r)
        if (run_off[r + 1] < run_off[r]) return fail(VBF_EINVAL, "run_off not nondecreasing at %u", r);
    const uint64_t total = run_off[nruns];
    if (total >= 0xFFFFFFFFull) return fail(VBF_EINVAL, "too many entries (%llu)", (unsigned long long)total);
    if (total && (!keys && offsets == nullptr)) return fail(VBF_EINVAL, "keys/offsets are NULL");
    if (total && (!offsets || !created || !tomb || !out_ids)) return fail(VBF_EINVAL, "NULL argument");
    if (map_n && (!map_keys || !map_off || !map_time)) return fail(VBF_EINVAL, "map arrays are NULL");
    if (total == 0) return VBF_OK;
    // merge levels: segment boundaries and per-pair tile starts per level, all uploaded at once
    const uint64_t tile = vbf::compact_tile();
    std::vector<uint64_t> bnd(run_off, run_off + nruns + 1);
    std::vector<uint64_t> all, tiles_all, ntiles_lv;
    std::vector<uint32_t> nseg_lv;
    uint64_t max_tiles = 1;
    uint32_t nseg = nruns;
    while (nseg > 1) {
        all.insert(all.end(), bnd.begin(), bnd.end());
        nseg_lv.push_back(nseg);
        uint64_t t = 0;
        for (uint32_t i = 0; i < nseg; i += 2) {
            tiles_all.push_back(t);
            const uint64_t len = bnd[std::min(i + 2, nseg)] - bnd[i];
            t += (len + tile - 1) / tile;
        }
        tiles_all.push_back(t);
        ntiles_lv.push_back(t);
        max_tiles = std::max(max_tiles, t);
        std::vector<uint64_t> nb;
        for (uint32_t i = 0; i < nseg; i += 2) nb.push_back(bnd[i]);
        nb.push_back(bnd[nseg]);
        bnd.swap(nb);
        nseg = (uint32_t)bnd.size() - 1;
    }
    size_t t1 = 0, t2 = 0, t3 = 0;
    HIP_TRY(vbf::select_u32(nullptr, &t1, nullptr, nullptr, nullptr, nullptr, total, s));
    HIP_TRY(vbf::select_i64(nullptr, &t2, nullptr, nullptr, nullptr, nullptr, total, s));
    t3 = std::max(t1, t2);
    const uint64_t o_pong = align256(total * 4), o_keep = o_pong + align256(total * 4);
    const uint64_t o_sel = o_keep + align256(total), o_upd = o_sel + align256(total * 4);
    const uint64_t o_ut = o_upd + align256(total), o_ro = o_ut + align256(total * 8);
    const uint64_t o_bnd = o_ro + align256((nruns + 1) * 8), o_tl = o_bnd + align256(all.size() * 8 + 8);
    const uint64_t o_pp = o_tl + align256(tiles_all.size() * 8 + 8), o_pq = o_pp + align256(total * 8);
    const uint64_t o_split = o_pq + align256(total * 8), o_misc = o_split + align256(max_tiles * 8);
    const uint64_t o_tmp = o_misc + 256, bytes = o_tmp + t3;
    void* ws = nullptr;
    int rc = get_workspace(s, bytes, &ws, kWsCompact);
    if (rc) return rc;
    char* b = static_cast<char*>(ws);
    uint32_t* ping = reinterpret_cast<uint32_t*>(b);
    uint32_t* pong = reinterpret_cast<uint32_t*>(b + o_pong);
    uint8_t* keep = reinterpret_cast<uint8_t*>(b + o_keep);
    uint32_t* sel = reinterpret_cast<uint32_t*>(b + o_sel);
    uint8_t* upd = reinterpret_cast<uint8_t*>(b + o_upd);
    int64_t* ut = reinterpret_cast<int64_t*>(b + o_ut);
    uint64_t* d_ro = reinterpret_cast<uint64_t*>(b + o_ro);
    uint64_t* d_bnd = reinterpret_cast<uint64_t*>(b + o_bnd);
    uint64_t* d_tl = reinterpret_cast<uint64_t*>(b + o_tl);
    uint64_t* pping = reinterpret_cast<uint64_t*>(b + o_pp);
    uint64_t* ppong = reinterpret_cast<uint64_t*>(b + o_pq);
    uint64_t* split = reinterpret_cast<uint64_t*>(b + o_split);
    uint64_t* misc = reinterpret_cast<uint64_t*>(b + o_misc);  // [0] n_out, [1] n_upd, [2] sort error
    HIP_TRY(hipMemcpyAsync(d_ro, run_off, (nruns + 1) * 8, hipMemcpyHostToDevice, s));
    if (!all.empty()) HIP_TRY(hipMemcpyAsync(d_bnd, all.data(), all.size() * 8, hipMemcpyHostToDevice, s));
    if (!tiles_all.empty())
        HIP_TRY(hipMemcpyAsync(d_tl, tiles_all.data(), tiles_all.size() * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(misc, 0, 16, s));
    HIP_TRY(hipMemsetAsync(misc + 2, 0xFF, 8, s));
    vbf::CompactArgs a{keys, offsets, created, tomb, d_ro, nruns, map_keys, map_off, map_time, map_n, use_ttl,
                       entry_ttl_ms, tomb_ttl_ms, now_ms, total};
    vbf::phase_begin(vbf::kPhaseMergeLevels, s);
    HIP_TRY(vbf::compact_check_sorted(a, reinterpret_cast<uint32_t*>(misc + 2), s));
    uint32_t* order = nullptr;
    uint64_t* opfx = nullptr;
    HIP_TRY(vbf::compact_merge_levels(a, d_bnd, d_tl, nseg_lv.data(), ntiles_lv.data(), (uint32_t)nseg_lv.size(),
                                      ping, pong, pping, ppong, split, &order, &opfx, s));
    vbf::phase_end(vbf::kPhaseMergeLevels, s);
    vbf::phase_begin(vbf::kPhaseFold, s);
    HIP_TRY(vbf::compact_fold(a, order, opfx, total, keep, sel, upd, ut, s));
    vbf::phase_end(vbf::kPhaseFold, s);
    vbf::phase_begin(vbf::kPhaseSelect, s);
    size_t tb = t3;
    HIP_TRY(vbf::select_u32(b + o_tmp, &tb, sel, keep, out_ids, misc, total, s));
    if (upd_ids && upd_time) {
        tb = t3;
        HIP_TRY(vbf::select_u32(b + o_tmp, &tb, order, upd, upd_ids, misc + 1, total, s));
        tb = t3;
        HIP_TRY(vbf::select_i64(b + o_tmp, &tb, ut, upd, upd_time, misc + 1, total, s));
    }
    vbf::phase_end(vbf::kPhaseSelect, s);
    uint64_t hv[3];
    HIP_TRY(hipMemcpyAsync(hv, misc, 24, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint32_t bad = (uint32_t)hv[2];
    if (bad != 0xFFFFFFFFu)
        return fail(VBF_EINVAL, "run entries not strictly increasing at entry %u (tables are SkipMaps)", bad);
    *n_out = hv[0];
    if (n_upd) *n_upd = (upd_ids && upd_time) ? hv[1] : 0;
    return VBF_OK;
}

int gather_entries(const uint8_t* keys, const uint64_t* offsets, const int64_t* created, const uint8_t* tomb,
                   const uint32_t* val, const uint32_t* ids, uint64_t n, uint8_t* out_keys, uint64_t out_keys_cap,
                   uint64_t* out_offsets, int64_t* out_created, uint8_t* out_tomb, uint32_t* out_val,
                   uint64_t* key_bytes, hipStream_t s) {
    if (!out_offsets) return fail(VBF_EINVAL, "out_offsets is NULL");
    if (n && (!offsets || !ids)) return fail(VBF_EINVAL, "NULL argument");
    if ((out_created && !created) || (out_tomb && !tomb) || (out_val && !val))
        return fail(VBF_EINVAL, "an output array without its input");
    size_t tmpb = 0;
    HIP_TRY(vbf::scan_u64(nullptr, &tmpb, nullptr, nullptr, n + 1, s));
    const uint64_t o_tmp = align256((n + 1) * 8);
    void* ws = nullptr;
    int rc = get_workspace(s, o_tmp + tmpb, &ws, kWsGather);
    if (rc) return rc;
    uint64_t* lens = static_cast<uint64_t*>(ws);
    HIP_TRY(vbf::gather_lens(offsets, ids, n, lens, s));
    HIP_TRY(vbf::scan_u64(static_cast<char*>(ws) + o_tmp, &tmpb, lens, out_offsets, n + 1, s));
    uint64_t total = 0;
    HIP_TRY(hipMemcpyAsync(&total, out_offsets + n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (key_bytes) *key_bytes = total;
    if (total > out_keys_cap || (total && !out_keys))
        return fail(VBF_EINVAL, "out_keys holds %llu < %llu bytes", (unsigned long long)out_keys_cap,
                    (unsigned long long)total);
    vbf::GatherArgs g{keys, offsets, created, tomb, val, ids, n, out_keys, out_offsets, out_created, out_tomb, out_val};
    HIP_TRY(vbf::gather(g, s));
    return VBF_OK;
}
}  // namespace

extern "C" {

int vbf_compact_merge_dev(const uint8_t* keys, const uint64_t* offsets, const int64_t* created_ms,
                          const uint8_t* tombstones, const uint64_t* run_off, uint32_t nruns, const uint8_t* map_keys,
                          const uint64_t* map_off, const int64_t* map_time, uint64_t map_n, int use_ttl,
                          uint64_t entry_ttl_ms, uint64_t tombstone_ttl_ms, uint64_t now_ms, uint32_t* out_ids,
                          uint64_t* n_out, uint32_t* upd_ids, int64_t* upd_time, uint64_t* n_upd, void* stream) {
    FORK_GUARD();
    int rc = compact_merge(keys, offsets, created_ms, tombstones, run_off, nruns, map_keys, map_off, map_time, map_n,
                           use_ttl, entry_ttl_ms, tombstone_ttl_ms, now_ms, out_ids, n_out, upd_ids, upd_time, n_upd,
                           (hipStream_t)stream);
    return rc ? rc : ok();
}

int vbf_gather_entries_dev(const uint8_t* keys, const uint64_t* offsets, const int64_t* created_ms,
                           const uint8_t* tombstones, const uint32_t* val_offsets, const uint32_t* ids, uint64_t n,
                           uint8_t* out_keys, uint64_t out_keys_cap, uint64_t* out_offsets, int64_t* out_created_ms,
                           uint8_t* out_tombstones, uint32_t* out_val_offsets, uint64_t* key_bytes, void* stream) {
    FORK_GUARD();
    int rc = gather_entries(keys, offsets, created_ms, tombstones, val_offsets, ids, n, out_keys, out_keys_cap,
                            out_offsets, out_created_ms, out_tombstones, out_val_offsets, key_bytes, (hipStream_t)stream);
    return rc ? rc : ok();
}

int vbf_compact_merge_host(const uint8_t* keys, const uint64_t* offsets, const int64_t* created_ms,
                           const uint8_t* tombstones, const uint64_t* run_off, uint32_t nruns, const uint8_t* map_keys,
                           const uint64_t* map_off, const int64_t* map_time, uint64_t map_n, int use_ttl,
                           uint64_t entry_ttl_ms, uint64_t tombstone_ttl_ms, uint64_t now_ms, uint32_t* out_ids,
                           uint64_t* n_out, uint32_t* upd_ids, int64_t* upd_time, uint64_t* n_upd, int device) {
    if (!n_out) return fail(VBF_EINVAL, "n_out is NULL");
    *n_out = 0;
    if (n_upd) *n_upd = 0;
    if (!nruns) return ok();
    if (!run_off) return fail(VBF_EINVAL, "run_off is NULL");
    const uint64_t total = run_off[nruns];
    if (total && (!offsets || !created_ms || !tombstones || !out_ids)) return fail(VBF_EINVAL, "NULL argument");
    if (map_n && (!map_keys || !map_off || !map_time)) return fail(VBF_EINVAL, "map arrays are NULL");
    DEVICE_SCOPE(device);
    hipStream_t s;
    int rc = filter_stream(device, &s);
    if (rc) return rc;
    const uint64_t kb = total ? offsets[total] : 0, mkb = map_n ? map_off[map_n] : 0;
    const uint64_t o_off = align256(kb), o_cr = o_off + align256((total + 1) * 8), o_tb = o_cr + align256(total * 8);
    const uint64_t o_mk = o_tb + align256(total), o_mo = o_mk + align256(mkb), o_mt = o_mo + align256((map_n + 1) * 8);
    const uint64_t o_ids = o_mt + align256(map_n * 8), o_ui = o_ids + align256(total * 4);
    const uint64_t o_ut = o_ui + align256(total * 4), bytes = o_ut + align256(total * 8);
    void* ws = nullptr;
    if ((rc = get_workspace(s, bytes, &ws, kWsCompactIn))) return rc;
    char* b = static_cast<char*>(ws);
    if (kb) HIP_TRY(hipMemcpyAsync(b, keys, kb, hipMemcpyHostToDevice, s));
    if (total) {
        HIP_TRY(hipMemcpyAsync(b + o_off, offsets, (total + 1) * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(b + o_cr, created_ms, total * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(b + o_tb, tombstones, total, hipMemcpyHostToDevice, s));
    }
    if (map_n) {
        if (mkb) HIP_TRY(hipMemcpyAsync(b + o_mk, map_keys, mkb, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(b + o_mo, map_off, (map_n + 1) * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(b + o_mt, map_time, map_n * 8, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    const bool want_upd = upd_ids && upd_time;
    uint64_t nu = 0;
    rc = compact_merge(reinterpret_cast<const uint8_t*>(b), reinterpret_cast<const uint64_t*>(b + o_off),
                       reinterpret_cast<const int64_t*>(b + o_cr), reinterpret_cast<const uint8_t*>(b + o_tb), run_off,
                       nruns, map_n ? reinterpret_cast<const uint8_t*>(b + o_mk) : nullptr,
                       map_n ? reinterpret_cast<const uint64_t*>(b + o_mo) : nullptr,
                       map_n ? reinterpret_cast<const int64_t*>(b + o_mt) : nullptr, map_n, use_ttl, entry_ttl_ms,
                       tombstone_ttl_ms, now_ms, reinterpret_cast<uint32_t*>(b + o_ids), n_out,
                       want_upd ? reinterpret_cast<uint32_t*>(b + o_ui) : nullptr,
                       want_upd ? reinterpret_cast<int64_t*>(b + o_ut) : nullptr, &nu, s);
    if (rc) return rc;
    if (*n_out) HIP_TRY(hipMemcpyAsync(out_ids, b + o_ids, *n_out * 4, hipMemcpyDeviceToHost, s));
    if (want_upd && nu) {
        HIP_TRY(hipMemcpyAsync(upd_ids, b + o_ui, nu * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(upd_time, b + o_ut, nu * 8, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (n_upd) *n_upd = nu;
    return ok();
}

}  // extern "C"
