// vbf_kernels.hpp -- internal launch interface between the C ABI (vbf_api.hip) and the kernels.
#pragma once

// Ablation builds (timing experiments, tools/ablate*.py): compiled with -DVBF_ABLATION_BUILD=1 and
// loaded through VBF_LIB, they honour VBF_ABLATE, which skips phases and so gives WRONG
// results.  The product library is built without it and ignores VBF_ABLATE.
#ifndef VBF_ABLATION_BUILD
#define VBF_ABLATION_BUILD 0
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vbf {

// A batch of keys resident in device memory.
//   offsets == nullptr : key j = keys[j*stride .. j*stride + stride)
//   offsets != nullptr : key j = keys[offsets[j]-off_base .. offsets[j+1]-off_base)
struct KeyBatch {
    const uint8_t* keys;
    const uint64_t* offsets;
    uint64_t off_base;
    uint64_t stride;
    uint64_t n;
    bool len_prefix;  // prepend LE64(len) (Rust `Hash for [u8]`)
};

hipError_t launch_build(const KeyBatch& kb, uint32_t m, uint32_t k, uint32_t* words, hipStream_t s);

// Optional per-phase timing (vbf_profile_*): HIP events recorded on the launch stream.
enum Phase { kPhaseTileSort = 0, kPhaseTranspose = 1, kPhaseSegOr = 2, kPhaseAtomicBuild = 3,
             kPhaseProbe = 4, kPhaseSstWalk = 5, kPhaseSstScan = 6, kPhaseSstEmit = 7,
             kPhaseMergeLevels = 8, kPhaseFold = 9, kPhaseSelect = 10, kPhaseProbePack = 11,
             kPhaseProbeSeg = 12, kPhaseProbeOut = 13, kNumPhases = 14 };
void phase_begin(int phase, hipStream_t s);
void phase_end(int phase, hipStream_t s);

// Partitioned build (vbf_partition.hip).  Key batches are processed in chunks of at most
// kBuildChunkIdx (build) / kPartChunkIdx (probe) bit indices; the workspace holds one chunk's
// sorted tiles + offset tables (build: 2.5 B per index, ~10.7 GB at 2^32; probe: 4 B per index).
// Each build chunk re-reads and re-writes the whole filter in k_seg_or, so build chunks are big:
// 2^32 holds config 5's 1B keys x k = 4 in one chunk (26.9 -> 26.5 ms: one k_seg_or pass over
// the 512 MiB filter instead of two, and that one fresh; profiles/r05/ab_cfg5_single_chunk.txt).
constexpr uint64_t kPartChunkIdx = 1ull << 30;
constexpr uint64_t kBuildChunkIdx = 1ull << 32;
bool partition_supported(uint32_t m, uint32_t k);
// chunk_idx: bit indices per build chunk (0: kBuildChunkIdx or VBF_BUILD_CHUNK_LOG2); the C ABI
// halves it when the workspace for the default chunk cannot be allocated (2^32
// indices take ~10.7 GB)
uint64_t build_chunk_default();
uint64_t partition_workspace_bytes(uint64_t n, uint32_t m, uint32_t k, uint64_t chunk_idx = 0);
// Partitioned probe (vbf_partition.hip): out (answer bytes) or count (hits), one of them.
bool probe_partition_supported(uint32_t m, uint32_t k);
uint64_t probe_workspace_bytes(uint64_t n, uint32_t m, uint32_t k);
hipError_t launch_probe_partitioned(const KeyBatch& kb, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
                                    unsigned long long* count, void* ws, uint64_t ws_bytes, hipStream_t s);
uint64_t probe_count_partials(uint64_t n, uint32_t m, uint32_t k);
// fresh: `words` holds no filter yet; the first chunk's segment pass writes every word without
// reading it (callers zero the words themselves where that pass cannot own every segment).
hipError_t launch_build_partitioned(const KeyBatch& kb, uint32_t m, uint32_t k, uint32_t* words,
                                    void* ws, uint64_t ws_bytes, bool atomic_merge, hipStream_t s,
                                    bool fresh = false, uint64_t chunk_idx = 0);
// Whether a fresh build of n keys can skip the zero fill (one chunk, one workgroup per segment).
bool partition_fresh_ok(uint64_t n, uint32_t m, uint32_t k, uint64_t chunk_idx = 0);
hipError_t launch_probe(const KeyBatch& kb, uint32_t m, uint32_t k, const uint32_t* words,
                        uint8_t* out, hipStream_t s);
// Count: `partial` holds count_partials(n) u32 of scratch; the hits are added to *count.
uint64_t count_partials(uint64_t n);
hipError_t launch_count(const KeyBatch& kb, uint32_t m, uint32_t k, const uint32_t* words,
                        unsigned long long* count, uint32_t* partial, hipStream_t s);
hipError_t launch_count_finish(const uint32_t* partial, uint64_t np, unsigned long long* count, hipStream_t s);
hipError_t launch_hashes(const KeyBatch& kb, uint32_t k, uint64_t* out, hipStream_t s);
hipError_t launch_or_words(uint32_t* dst, const uint32_t* src, uint64_t nwords, hipStream_t s);
hipError_t launch_popcount(const uint32_t* words, uint64_t nwords, unsigned long long* out,
                           hipStream_t s);
hipError_t launch_gen_fixed(uint64_t seed, uint64_t base, uint64_t n, uint32_t len, uint8_t* out,
                            hipStream_t s);
hipError_t launch_gen_var(uint64_t seed, uint64_t base, uint64_t n, const uint64_t* offsets,
                          uint8_t* out, hipStream_t s);


// SST data.db decode (vbf_sst.hip).  Output arrays may be NULL.
struct SstArgs {
    const uint8_t* data;
    uint64_t len;
    const uint32_t* blocks;  // block start offsets (index.db)
    uint64_t nblocks;
    uint32_t* counts;        // [nblocks + 1] entry counts (walk pass)
    uint16_t* pos;           // [nblocks * 256] entry starts within each block (walk pass)
    uint32_t* lmin;          // [nblocks] shortest / longest key per block (walk pass)
    uint32_t* lmax;
    const uint64_t* ebase;   // [nblocks + 1] exclusive scan of counts (emit pass)
    uint8_t* keys;
    uint64_t* offsets;       // [n + 1] absolute positions in keys
    uint32_t* val_off;
    uint64_t* created;
    uint8_t* tomb;
    uint32_t* err;           // [0] error bits, [1] first bad block, [2]/[3] min/max key length
    uint32_t ablate;         // timing experiments only (VBF_ABLATE 11-14, ablation builds)
    uint32_t walk_v;         // 1: vector-register entry walk (default), 0: scalar (VBF_SST_WALK)
};
hipError_t sst_count(const SstArgs& a, hipStream_t s);
hipError_t sst_emit(const SstArgs& a, hipStream_t s);
uint64_t sst_pos_bytes(uint64_t nblocks);
hipError_t sst_len_range(const uint32_t* lmin, const uint32_t* lmax, uint64_t nblocks, uint32_t* out2, void* tmp,
                         size_t* tmp_bytes, hipStream_t s);
hipError_t sst_scan(const uint32_t* counts, uint64_t* ebase, uint64_t nblocks, void* tmp, size_t* tmp_bytes,
                    hipStream_t s);
// Batched probe across SSTs (vbf_multi.hip).
struct MultiSst {
    const uint32_t* words;
    uint64_t m, mu;
    uint32_t k, col;                          // col: the SST's column in `out`
    uint64_t lo_beg, lo_end, hi_beg, hi_end;  // smallest / biggest key in `bounds`
};
struct MultiArgs {
    const uint8_t* keys;
    const uint64_t* offsets;
    uint64_t off_base, stride, n;
    uint32_t nsst;          // table entries
    const MultiSst* tab;    // device table, nsst entries
    const uint8_t* bounds;  // device, NULL = no key-range test
    uint8_t* out;           // n rows of out_stride bytes
    uint32_t* err;          // device word: set to 1 when a key reaches a filter with m == 0 < k
    uint32_t out_stride;    // all SSTs of the call
};
hipError_t launch_multi_probe(const MultiArgs& a, bool len_prefix, hipStream_t s);
// Interleaved groups (vbf_multi_part.hip): G <= 8 filters of one (m, k) probed together, their bits
// interleaved into one byte per position; a partitioned probe tests all G per entry.
constexpr uint32_t kMaxGroup = 8;
struct MultiGroup {
    const uint32_t* words[kMaxGroup];
    uint32_t G, k;
    uint64_t m;
    uint32_t col[kMaxGroup];
    uint64_t lo_beg[kMaxGroup], lo_end[kMaxGroup], hi_beg[kMaxGroup], hi_end[kMaxGroup];
};
bool multi_group_supported(uint64_t m, uint32_t k);
uint64_t multi_group_workspace_bytes(uint64_t n, uint64_t m, uint32_t k);
hipError_t launch_multi_probe_group(const KeyBatch& kb, const MultiGroup& g, const uint8_t* bounds, uint8_t* out,
                                    uint32_t out_stride, void* ws, uint64_t ws_bytes, hipStream_t s);
// Compaction merge (vbf_compact.hip).
struct CompactArgs {
    const uint8_t* keys;
    const uint64_t* offsets;  // arena: entry e = keys[offsets[e] .. offsets[e+1])
    const int64_t* created;   // ms
    const uint8_t* tomb;
    const uint64_t* run_off;  // device, nruns + 1 entry boundaries (run_off[0] = 0)
    uint32_t nruns;
    const uint8_t* map_keys;  // tombstone map: sorted unique keys
    const uint64_t* map_off;
    const int64_t* map_time;
    uint64_t map_n;
    int use_ttl;
    uint64_t entry_ttl_ms, tomb_ttl_ms, now_ms;
    uint64_t run_off_host_total;  // entries in all runs (host side)
};
struct GatherArgs {
    const uint8_t* keys;
    const uint64_t* offsets;
    const int64_t* created;
    const uint8_t* tomb;
    const uint32_t* val;
    const uint32_t* ids;
    uint64_t n;
    uint8_t* out_keys;
    const uint64_t* out_off;
    int64_t* out_created;
    uint8_t* out_tomb;
    uint32_t* out_val;
};
hipError_t launch_iota_u32(uint32_t* out, uint64_t n, hipStream_t s);
hipError_t compact_check_sorted(const CompactArgs& a, uint32_t* err, hipStream_t s);
hipError_t compact_merge_levels(const CompactArgs& a, const uint64_t* d_bnd_all, const uint64_t* d_tiles_all,
                                const uint32_t* nseg_per_level, const uint64_t* ntiles_per_level, uint32_t nlevels,
                                uint32_t* ping, uint32_t* pong, uint64_t* pping, uint64_t* ppong, uint64_t* split,
                                uint32_t** result, uint64_t** presult, hipStream_t s);
uint32_t compact_tile();
hipError_t compact_fold(const CompactArgs& a, const uint32_t* order, const uint64_t* opfx, uint64_t total,
                        uint8_t* keep, uint32_t* sel, uint8_t* upd, int64_t* upd_time, hipStream_t s);
hipError_t select_u32(void* tmp, size_t* bytes, const uint32_t* in, const uint8_t* flags, uint32_t* out,
                      uint64_t* nsel, uint64_t n, hipStream_t s);
hipError_t select_i64(void* tmp, size_t* bytes, const int64_t* in, const uint8_t* flags, int64_t* out,
                      uint64_t* nsel, uint64_t n, hipStream_t s);
hipError_t gather_lens(const uint64_t* offsets, const uint32_t* ids, uint64_t n, uint64_t* lens, hipStream_t s);
hipError_t scan_u64(void* tmp, size_t* bytes, const uint64_t* in, uint64_t* out, uint64_t n, hipStream_t s);
hipError_t gather(const GatherArgs& g, hipStream_t s);
hipError_t gen_sst_fixed(uint64_t seed, uint64_t base, uint64_t n, uint32_t len, uint8_t* data, uint32_t* blocks,
                         hipStream_t s);
}  // namespace vbf
