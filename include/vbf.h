/*
 * vbf.h -- C ABI of the MI355X (gfx950) Bloom-filter engine behind velarixdb's src/filter.
 *
 * This is the drop-in boundary.  Every entry point takes plain pointers and sizes, never
 * aborts or throws across the ABI, and returns an int status (VBF_OK = 0) unless noted.
 * The message of the last failure on the calling thread is available from vbf_last_error().
 *
 * Reference interface replaced (velarixdb 0.0.17, /root/reference):
 *   BloomFilter struct                 src/filter/bf.rs:38-58      -> vbf_filter (opaque handle)
 *   BloomFilter::new                   src/filter/bf.rs:62-81      -> vbf_filter_new / vbf_size
 *   BloomFilter::set                   src/filter/bf.rs:84-92      -> vbf_filter_set_host / _dev
 *   BloomFilter::contains              src/filter/bf.rs:95-105     -> vbf_filter_contains_host / _dev
 *   BloomFilter::build_filter_from_entries src/filter/bf.rs:126-128 -> vbf_filter_set_host (batch)
 *                                                                     / vbf_filter_set_host_async
 *   BloomFilter::recover_meta          src/filter/bf.rs:135-150    -> vbf_filter_recover
 *   BloomFilter::serialize             src/filter/bf.rs:158-172    -> vbf_filter_serialize
 *   BloomFilter::write + recover_meta + lazy rebuild, bits persisted (bf.rs:114-150,
 *     range.rs:117-128)                                            -> vbf_filter_serialize_ext / _recover_ext
 *   FilterFileNode::recover            src/fs/mod.rs:768-796       -> vbf_meta_parse
 *   BloomFilter::clear                 src/filter/bf.rs:180-195    -> vbf_filter_clear
 *   num_elements / num_bits / num_of_hash_functions bf.rs:198-213  -> vbf_filter_num_*
 *   calculate_hash                     src/filter/bf.rs:222-227    -> vbf_hashes_dev (parity)
 *   calculate_no_of_bits               src/filter/bf.rs:230-233    -> vbf_num_bits
 *   calculate_no_of_hash_function      src/filter/bf.rs:236-239    -> vbf_num_hash_functions
 *   Clone (shares the bit array)       src/filter/bf.rs:242-254    -> vbf_filter_clone
 *   Default                            src/filter/bf.rs:256-267    -> vbf_filter_default
 *   DataFileNode::load_entries         src/fs/mod.rs:275-332       -> vbf_sst_decode_dev / _host
 *   index.db block offsets             src/index/indexer.rs:151-170 -> vbf_sst_index_blocks
 *   lazy filter rebuild                src/key_range/range.rs:117-128 -> vbf_filter_rebuild_from_sst_*
 *   KeyRange::filter_sstables_by_key_range src/key_range/range.rs:91-147 -> vbf_multi_probe_* (batch)
 *   SizedTierRunner::merge_ssts_in_buckets src/compactors/sized.rs:170-320 -> vbf_compact_merge_*
 *
 * Key batches.  `keys` holds the key bytes back to back.  When `offsets` is non-NULL it has
 * n+1 nondecreasing entries and key j is keys[offsets[j] .. offsets[j+1]) (positions are
 * absolute in `keys`; offsets[0] need not be 0); otherwise key j is
 * keys[j*stride .. (j+1)*stride).  Offsets live where the keys live (device or host).  `len_prefix` = 1 hashes LE64(len) || key, which is
 * Rust's `Hash for [u8]` / `Vec<u8>` (every production call site: memtable/mem.rs:209-210,224,
 * key_range/range.rs:130,136,171, filter/bf.rs:127).  len_prefix = 0 hashes the bytes as given,
 * for callers that pre-encode other Hash impls (usize -> 8 LE bytes, as bf.rs's tests use).
 *
 * Filter words.  ceil(m/32) uint32 words, bit i = words[i/32] bit (i%32): the storage of
 * bit-vec 0.6.3 `BitVec<u32>` (Cargo.toml:19).  Builds OR into existing bits, never clear.
 */
#ifndef VBF_H
#define VBF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VBF_OK 0
#define VBF_EINVAL (-1)   /* bad argument (where the reference asserts: bf.rs:63-67)    */
#define VBF_EHIP (-2)     /* HIP runtime / launch failure                               */
#define VBF_ENOMEM (-3)   /* device or pinned-host allocation failed                    */
#define VBF_ENODEV (-4)   /* no usable gfx950 device                                    */
#define VBF_EDIVZERO (-5) /* m == 0 with k > 0: the reference panics (`% 0`, bf.rs:88)   */

/* `device` of a filter whose bits live in host memory (see "Residency" below). */
#define VBF_DEVICE_HOST (-1)
/* `device` for vbf_filter_new, _new_sized, _default, _recover, _recover_ext and _migrate: the library places the filter,
 * round-robin over the visible devices (successive filters land on different GPUs). */
#define VBF_DEVICE_AUTO (-2)

const char* vbf_version(void);
const char* vbf_last_error(void); /* thread-local; "" when the last call succeeded */
int vbf_device_count(int* count);

/* Kernel-phase timing with hipEvents on the launch streams (for bench.py's roofline):
 * phases 0 tile-sort, 1 transpose, 2 segment-OR (partitioned build), 3 atomic build, 4 probe,
 * 5 data.db walk, 6 data.db scan, 7 data.db emit, 8 compaction merge levels, 9 fold, 10 select,
 * 11 partitioned-probe pack, 12 probe segment test, 13 probe answers.
 * vbf_profile_read synchronizes, returns per-phase summed ms and launch counts, and resets. */
int vbf_profile_enable(int on);
int vbf_profile_read(double* ms, uint64_t* launches, int nphases);

/* ---- sizing (host arithmetic, glibc log, Rust `as u32` saturation) ---- */
uint32_t vbf_num_bits(uint64_t n, double p);              /* bf.rs:230-233 */
uint32_t vbf_num_hash_functions(uint32_t m, uint32_t n);  /* bf.rs:236-239 */
/* bf.rs:62-70: asserts p >= 0 and n > 0 (-> VBF_EINVAL), m = num_bits(n, p),
 * k = num_hash_functions(m, n as u32). */
int vbf_size(double p, uint64_t n, uint32_t* m, uint32_t* k);

/* ---- filter.db metadata: u32 k | u32 n | f64 p, little-endian, 16 bytes ---- */
void vbf_meta_serialize(uint32_t k, uint32_t n, double p, uint8_t out[16]); /* bf.rs:158-172 */
int vbf_meta_parse(const uint8_t* in, size_t len, uint32_t* k, uint32_t* n, double* p); /* fs/mod.rs:768-796 */

/* ---- stateless kernels on device-resident buffers; `stream` is a hipStream_t (NULL = the
 *      legacy default stream).  Calls are asynchronous on that stream. ---- */
int vbf_build_dev(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                  int len_prefix, uint32_t m, uint32_t k, uint32_t* words, void* stream);
int vbf_probe_dev(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                  int len_prefix, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
                  void* stream);
/* Build strategies.  ATOMIC: one lane per key, k global atomicOr's per key.  PARTITIONED:
 * hash + per-tile LDS sort by 2^20-bit segment, then one workgroup ORs each segment in LDS
 * (no global atomics; needs 1 <= k <= 32 and a device workspace the library caches per
 * stream).  AUTO picks PARTITIONED for batches of >= 2^22 bit indices.  Results are
 * bit-identical.  vbf_build_dev/_ex expect stream-ordered exclusive use of `words` (the
 * partitioned path rewrites whole segments); the host and handle APIs merge atomically. */
#define VBF_BUILD_AUTO 0
#define VBF_BUILD_ATOMIC 1
#define VBF_BUILD_PARTITIONED 2
/* OR into a build strategy: `words` holds no filter yet -- BloomFilter::new (bf.rs:62-81, an
 * all-zero BitVec) fused with build_filter_from_entries (bf.rs:126-128), as flush and compaction
 * call them.  Every one of the ceil(m/32) words is written (prior contents ignored, the bits of
 * keys set, all others 0), with no separate zero fill: the partitioned build's segment pass
 * writes its segments without reading them first.  Without the flag a build ORs into `words`. */
#define VBF_BUILD_FRESH 0x100
int vbf_build_dev_ex(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                     int len_prefix, uint32_t m, uint32_t k, uint32_t* words, int strategy,
                     void* stream);
/* Device bytes the partitioned build of n keys needs as workspace (0 if unsupported): the tile
 * image (~2.6 bytes per bit index) and the run ends of one build chunk of up to 2^32 bit indices
 * -- about 11 GB for a chunk of 2^32 indices (config 5's 1B keys at k = 4), kept per stream until
 * vbf_release_workspaces.  When that allocation fails the build retries with half the chunk, down
 * to 2^28 indices (VBF_WS_MAX_BYTES caps the workspace the same way). */
uint64_t vbf_build_workspace_bytes(uint64_t n, uint32_t m, uint32_t k);
/* Free every cached workspace (synchronizes the streams that own them). */
int vbf_release_workspaces(void);
/* Adds the number of keys the filter answers "present" for to *count_dev (device u64). */
int vbf_probe_count_dev(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                        int len_prefix, uint32_t m, uint32_t k, const uint32_t* words,
                        unsigned long long* count_dev, void* stream);

/* Same with an explicit strategy: VBF_BUILD_ATOMIC (one lane per key, early exit on the first
 * clear bit, random filter loads), VBF_BUILD_PARTITIONED (keys hashed in tiles, entries sorted by
 * 2^20-bit filter segment, every bit test against a segment staged in LDS; all k hashes per key),
 * VBF_BUILD_AUTO (the calls above): for batches of >= 2^24 bit tests against filters of >= 2^26
 * bits it probes the first 65 536 keys by gather, reads their hit count back (one stream
 * synchronisation) and goes partitioned when >= 35 % hit (positive sweeps), gather otherwise.
 * Identical answers either way. */
int vbf_probe_dev_ex(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                     int len_prefix, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
                     int strategy, void* stream);
int vbf_probe_count_dev_ex(const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
                           uint64_t n, int len_prefix, uint32_t m, uint32_t k,
                           const uint32_t* words, unsigned long long* count_dev, int strategy,
                           void* stream);
/* out[j*k + i] = calculate_hash(key_j, i) (bf.rs:222-227). */
int vbf_hashes_dev(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                   int len_prefix, uint32_t k, uint64_t* out, void* stream);
/* dst |= src over nwords (16-byte aligned): merging partial filters of one key set. */
int vbf_or_words_dev(uint32_t* dst, const uint32_t* src, uint64_t nwords, void* stream);
/* dst[i] = OR over p < nparts of src[p * part_stride + i], i < nwords, in one pass (the fold of the
 * multi-GPU OR all-reduce: every rank's copy of one bit range, received back to back; the bitwise
 * OR that merges partial filters of one key set, bf.rs:89).  16-byte aligned pointers, part_stride
 * a multiple of 4 words and >= nwords; dst may be src (part 0) itself. */
int vbf_or_fold_dev(uint32_t* dst, const uint32_t* src, uint64_t nwords, uint32_t nparts, uint64_t part_stride,
                    void* stream);
/* *count_dev += popcount(words[0..nwords)). */
int vbf_popcount_dev(const uint32_t* words, uint64_t nwords, unsigned long long* count_dev,
                     void* stream);

/* ---- synthetic key sets (benchmarks/tests; definitions in DESIGN.md, section Workloads) ---- */
int vbf_gen_fixed_dev(uint64_t seed, uint64_t base, uint64_t n, uint32_t len, uint8_t* out,
                      void* stream);
int vbf_gen_var_dev(uint64_t seed, uint64_t base, uint64_t n, const uint64_t* offsets,
                    uint8_t* out, void* stream);

/* ---- one-shot host-pointer variants: keys/words in host memory, chunked H2D through pinned
 *      staging on `device`, synchronous.  Build ORs into `words` (nwords = ceil(m/32)). ---- */
int vbf_build_host(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                   int len_prefix, uint32_t m, uint32_t k, uint32_t* words, uint64_t nwords,
                   int device);
int vbf_probe_host(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                   int len_prefix, uint32_t m, uint32_t k, const uint32_t* words, uint64_t nwords,
                   uint8_t* out, int device);

/* Compaction fan-in (src/compactors/sized.rs:170-200 builds one filter per merged SSTable, each
 * from its own entries): independent builds spread over devices[0..ndevices), shard s on
 * devices[s % ndevices], one host thread and its own staging streams per device, shards of one
 * device in order.  Each shard is a vbf_build_host call: host keys, ORed into its host words.
 * Per-shard status lands in shards[s].status; the return value is the first failure's (the
 * message is this thread's vbf_last_error). */
typedef struct vbf_shard {
    const uint8_t* keys;
    const uint64_t* offsets; /* n+1 host offsets, or NULL for fixed `stride` */
    uint64_t stride;
    uint64_t n;
    int len_prefix;
    uint32_t m, k;
    uint32_t* words;         /* host, ceil(m/32) words, OR-accumulated */
    uint64_t nwords;
    int status;              /* out */
} vbf_shard;
int vbf_build_shards_host(vbf_shard* shards, uint64_t nshards, const int* devices, int ndevices);

/* ---- BloomFilter handle: the bit array lives in HBM on `device` ----
 *
 * Residency.  A filter created on a device keeps its bits in that GPU's HBM: batch builds and
 * probes run as kernels, and every call on the filter is ordered after the filter's previous
 * one whatever stream either ran on (the reference's Mutex<BitVec>, bf.rs:85,96): a _dev call
 * is queued behind the last asynchronous operation on the filter, a host call waits for it.
 * A filter created with device = VBF_DEVICE_HOST keeps its bits in host memory and runs
 * set/contains on the CPU inside this library (same SipHash-1-3 rounds, Rust's `hash % m`):
 * the memtable's filter, one contains + set per put (memtable/mem.rs:207-221) and one contains
 * per get (:223-230), where a kernel launch per key would cost two PCIe round trips.  Such a
 * filter needs no GPU; the _dev, rebuild and multi-probe entry points reject it (VBF_EINVAL).
 * vbf_filter_migrate moves a filter's bits between host and devices in place (clones follow).
 *
 * Element count.  no_of_elements (bf.rs:46) lives in the handle only: set_host / set_dev /
 * rebuild add the number of keys, recover loads the stored n, clones copy it (bf.rs:248), and
 * vbf_filter_set_num_elements assigns it (bf.rs:143).  A binding keeps no second counter. */
typedef struct vbf_filter vbf_filter;

int vbf_filter_new(double p, uint64_t no_of_elements, int device, vbf_filter** out); /* bf.rs:62-81 */
int vbf_filter_default(int device, vbf_filter** out);                               /* bf.rs:256-267 */
/* A filter of exactly m bits and k hash functions (the struct's pub fields set directly,
 * bf.rs:38-58), no elements, false_positive_rate p. */
int vbf_filter_new_sized(uint32_t m, uint32_t k, double p, int device, vbf_filter** out);
/* recover_meta (bf.rs:135-150): k and n from the 16-byte metadata, m recomputed from n, bits 0. */
int vbf_filter_recover(const uint8_t* meta, size_t len, int device, vbf_filter** out);
int vbf_filter_clone(const vbf_filter* f, vbf_filter** out); /* shares the bit array, bf.rs:242-254 */
void vbf_filter_free(vbf_filter* f);

/* set over a batch (bf.rs:84-92 per key; build_filter_from_entries bf.rs:126-128).
 * no_of_elements += n (u32, wrapping like AtomicU32::fetch_add).  _host takes host keys (any
 * residency: a host-resident filter hashes them on the CPU, a device-resident one streams them
 * to its GPU); _dev takes device keys and a stream (device-resident filters only). */
int vbf_filter_set_host(vbf_filter* f, const uint8_t* keys, const uint64_t* offsets,
                        uint64_t stride, uint64_t n, int len_prefix);
int vbf_filter_set_dev(vbf_filter* f, const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
                       uint64_t n, int len_prefix, void* stream);
/* set over host keys, returning before the work is done (build_filter_from_entries for a
 * device-resident filter, bf.rs:126-128, without blocking the caller).  The batch is queued on
 * its device's worker thread, which streams it to the GPU exactly as vbf_filter_set_host does;
 * no_of_elements += n at once.  Every later call on the filter (or a clone) first waits for the
 * queued sets, so results are those of the synchronous call; a failure is returned by the next
 * call on the filter.  With `release` NULL the library copies the keys before returning (the
 * caller may reuse its buffers); otherwise it reads the caller's buffers and calls
 * release(release_ctx) from its worker once it no longer needs them (a Rust caller hands over
 * its packed Vec and drops it there).  Host-resident filters set synchronously (then release). */
int vbf_filter_set_host_async(vbf_filter* f, const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
                              uint64_t n, int len_prefix, void (*release)(void*), void* release_ctx);
/* Wait until every queued or in-flight operation on the filter has finished (returns a queued
 * set's failure).  vbf_filter_busy: 1 while such work is outstanding, 0 when idle, < 0 error. */
int vbf_filter_sync(vbf_filter* f);
int vbf_filter_busy(const vbf_filter* f);
/* Writers of the bits through vbf_filter_words_dev (an OR/merge kernel on the caller's stream)
 * bracket their work: vbf_filter_stream_wait makes `stream` wait for the filter's previous
 * operations, vbf_filter_stream_record makes the work queued on `stream` so far the filter's
 * last operation (later calls are ordered after it; the host mirror is refreshed behind it).
 * Every write through the pointer must be declared with vbf_filter_stream_record: once
 * vbf_filter_words_dev has handed the pointer out, the library no longer trusts its host mirror
 * (host reads copy the words from the GPU each time, and migrate copies instead of assuming the
 * words are zero) until the next vbf_filter_stream_record; a write made after that record and
 * not recorded itself may be missed by host-side reads.  A writer that skips stream_wait must
 * synchronize its stream before the next call on the filter.
 * A failed asynchronous set is returned once, by the next call on the filter that waits for
 * the queue (every call but vbf_filter_busy and the accessors).  `release` runs after the job
 * counts as done, so it may call back into the library.  A child forked while a set is queued
 * does not run it: the child's next call on that filter returns VBF_EINVAL.  More generally, HIP
 * does not survive fork(): in a child of a process that used the GPU through the library, every
 * call on a device-resident filter (and creating one) and every stateless device-pointer entry
 * point returns VBF_EINVAL before any HIP call, and freeing a handle there releases no device
 * memory (it is the parent's); host-resident filters work as usual. */
int vbf_filter_stream_wait(const vbf_filter* f, void* stream);
int vbf_filter_stream_record(vbf_filter* f, void* stream);
/* contains over a batch (bf.rs:95-105): out[j] = 1 when every one of the k bits is set.
 * Host mirror: a device-resident filter keeps a pinned host copy of its bits, refreshed after
 * device writes, and vbf_filter_contains_host / vbf_multi_probe_host batches of at most
 * VBF_MIRROR_MAX_KEYS (env, default 256) keys answer from it on the CPU -- the read path's one
 * contains per SST per get (key_range/range.rs:130,136,171) costs what it costs on a
 * host-resident filter instead of a PCIe round trip.  Larger batches run on the GPU. */
int vbf_filter_contains_host(const vbf_filter* f, const uint8_t* keys, const uint64_t* offsets,
                             uint64_t stride, uint64_t n, int len_prefix, uint8_t* out);
int vbf_filter_contains_dev(const vbf_filter* f, const uint8_t* keys, const uint64_t* offsets,
                            uint64_t stride, uint64_t n, int len_prefix, uint8_t* out, void* stream);

uint32_t vbf_filter_num_bits(const vbf_filter* f);           /* bf.rs:204-207 */
uint32_t vbf_filter_num_elements(const vbf_filter* f);       /* bf.rs:198-201 */
uint32_t vbf_filter_num_hash_functions(const vbf_filter* f); /* bf.rs:210-213 */
double vbf_filter_false_positive_rate(const vbf_filter* f);  /* bf.rs:54 */
int vbf_filter_device(const vbf_filter* f);          /* a device id or VBF_DEVICE_HOST */
/* Bytes of host memory the filter's bits hold: the host-resident words (allocated on their first
 * use, so a filter created on the host and migrated to a GPU before any set -- the compaction
 * filter of compactors/sized.rs:192-193 -- holds none) plus a device filter's pinned host mirror. */
uint64_t vbf_filter_host_bytes(const vbf_filter* f);
uint32_t* vbf_filter_words_dev(const vbf_filter* f); /* device pointer to the bit array (NULL if host) */
/* Read-only device pointer to the bit array (NULL if host-resident), e.g. the source of an OR
 * merge: unlike vbf_filter_words_dev it does not mark the bits externally written, so the host
 * mirror stays trusted.  Readers order themselves with vbf_filter_stream_wait. */
const uint32_t* vbf_filter_words_dev_read(const vbf_filter* f);
/* no_of_elements = n (bf.rs:143 assigns it on recover_meta). */
int vbf_filter_set_num_elements(vbf_filter* f, uint32_t n);
/* Binding bookkeeping kept in the handle, so a binding's BloomFilter struct needs no private
 * fields: velarixdb builds `BloomFilter { file_path: Some(..), ..Default::default() }` outside
 * filter::bf (db/recovery.rs:143-146, tests/workload.rs:309-312), which a private field would
 * forbid.  Both are per handle and copied by vbf_filter_clone, like the struct's plain fields
 * (bf.rs:242-254).
 * sst entries: the entry count of the SST this filter was batch-built from
 * (build_filter_from_entries), VBF_EXT_NONE until set; the binding's write() passes it to
 * vbf_filter_serialize_ext.  restored: vbf_filter_recover_ext loaded persisted bits;
 * vbf_filter_take_restored returns 1 once (and clears it), so the build_filter_from_entries that
 * follows recover_meta on the lazy-rebuild path (range.rs:117-128) can skip the rebuild. */
int vbf_filter_set_sst_entries(vbf_filter* f, uint64_t entries);
uint64_t vbf_filter_sst_entries(const vbf_filter* f);
int vbf_filter_take_restored(vbf_filter* f); /* 1 or 0; < 0 on error */
/* Move the (shared) bit array to `device` or to host memory (VBF_DEVICE_HOST), in place. */
int vbf_filter_migrate(vbf_filter* f, int device);
int vbf_filter_serialize(const vbf_filter* f, uint8_t out[16]); /* bf.rs:158-172 */
/* clear (bf.rs:180-195): zero this filter's (shared) bits and return a fresh empty filter with
 * the same m, k and p. */
int vbf_filter_clear(vbf_filter* f, vbf_filter** out);
/* Bit-array persistence: copy the ceil(m/32) words out / in. */
int vbf_filter_words_to_host(const vbf_filter* f, uint32_t* out, uint64_t nwords);
int vbf_filter_words_from_host(vbf_filter* f, const uint32_t* in, uint64_t nwords);

/* Host mirror mode (see contains above): OFF frees it and sends every contains to the GPU;
 * LAZY (default, env VBF_MIRROR) fills it with one D2H on the first small contains after a
 * device write; EAGER queues that D2H behind every device write, off the read path. */
#define VBF_MIRROR_OFF 0
#define VBF_MIRROR_LAZY 1
#define VBF_MIRROR_EAGER 2
int vbf_filter_set_mirror(vbf_filter* f, int mode);

/* filter.db with the bit array persisted after the reference's 16 bytes.
 * Layout (little-endian): the 16-byte header of vbf_filter_serialize (bf.rs:158-172), then
 *   u32 magic "VBFW" | u32 version 2 | u32 m | u32 nwords | u64 entries | u64 checksum | words
 * The reference reads exactly 16 bytes (fs/mod.rs:768-796), so the file stays readable by it.
 * The words are those recover_meta + build_filter_from_entries (range.rs:117-128) would rebuild:
 * a filter of m = num_bits(n_stored, p) bits (bf.rs:144-147) holding the SST's `entries` keys.
 *
 * vbf_filter_serialize_ext: `entries` = the SST's data.db entry count, or VBF_EXT_NONE for the
 * reference's 16 bytes alone.  When the filter's own m equals that recovery m (a compaction-built
 * filter, sized from its table's entries: sized.rs:192-193) its words are written; otherwise
 * (a memtable-born filter, sized from the write-buffer capacity: mem.rs:188-191) the recovery-
 * shaped words are built from `keys` (the SST's `entries` keys, layout as for set; on the CPU for
 * a host-resident filter, on its GPU otherwise), and with no keys only the 16 bytes are written.
 * *len = bytes needed; buf NULL is a size query; cap < *len is VBF_EINVAL.
 * vbf_filter_recover_ext: vbf_filter_recover, then, when the extension is present, intact
 * (checksum) and of the recovered m, loads its words and sets no_of_elements = n + entries
 * (what the rebuild leaves), *restored = 1: the caller skips the rebuild.  Otherwise
 * *restored = 0 and the caller rebuilds as the reference does. */
#define VBF_EXT_NONE UINT64_MAX
int vbf_filter_serialize_ext(const vbf_filter* f, const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
                             uint64_t entries, int len_prefix, uint8_t* buf, uint64_t cap, uint64_t* len);
int vbf_filter_recover_ext(const uint8_t* bytes, uint64_t len, int device, vbf_filter** out, int* restored);

/* Synthetic data.db (bench / tests): n entries whose keys are vbf_gen_fixed_dev's, value offset
 * (u32)j, created_at 1720785462000 + j ms, tombstone j % 97 == 0, blocked as
 * Table::write_to_file blocks them (src/sst/table.rs:295-324): floor(4096 / (len + 17)) entries
 * per block.  data: n * (len + 17) bytes; blocks: ceil(n / per_block) u32 start offsets. */
int vbf_gen_sst_fixed_dev(uint64_t seed, uint64_t base, uint64_t n, uint32_t len, uint8_t* data,
                          uint32_t* blocks, void* stream);

/* ---- SST data.db decode ----
 * data.db = blocks of whole entries, entry = u32 key_len | key | u32 value offset | i64
 * created_at ms | u8 tombstone (src/block/block_manager.rs:168-190), each block <= 4096 bytes
 * (:121-125); index.db holds one u32 key_len | key | u32 block offset record per block
 * (src/index/indexer.rs:151-170).  The decode is block-parallel, so it needs the block offsets. */

/* index.db bytes -> block start offsets.  Writes min(cap, count) offsets (offsets may be NULL)
 * and the count to *nblocks; VBF_EINVAL on a truncated record.  Host-only. */
int vbf_sst_index_blocks(const uint8_t* index, uint64_t len, uint32_t* offsets, uint64_t cap,
                         uint64_t* nblocks);

/* DataFileNode::load_entries (src/fs/mod.rs:275-332) on the device.  data/blocks are device
 * pointers; outputs are device pointers, each may be NULL: keys (packed key bytes, 4-byte aligned,
 * keys_cap >= len - 17 n), offsets (n+1 absolute positions in keys: the build's key layout),
 * val_offsets, created_ms, tombstones (1 iff the byte is 1, as the reference reads it),
 * entries_cap >= n (+1 for offsets).  *n_out = entry count, also when the outputs are too small
 * (VBF_EINVAL) so a first call with NULL outputs sizes them.  Synchronizes the stream once (the
 * entry count); the output pass is left queued on it.  A malformed file (entry crossing its block,
 * offsets out of order) is VBF_EINVAL, where the reference reports UnexpectedEof. */
int vbf_sst_decode_dev(const uint8_t* data, uint64_t len, const uint32_t* blocks, uint64_t nblocks,
                       uint8_t* keys, uint64_t keys_cap, uint64_t* offsets, uint32_t* val_offsets,
                       uint64_t* created_ms, uint8_t* tombstones, uint64_t entries_cap,
                       uint64_t* n_out, void* stream);

/* Same from host buffers (the data.db and index.db file contents) to host outputs; decoded on
 * `device`.  Synchronous. */
int vbf_sst_decode_host(const uint8_t* data, uint64_t len, const uint8_t* index, uint64_t index_len,
                        uint8_t* keys, uint64_t keys_cap, uint64_t* offsets, uint32_t* val_offsets,
                        uint64_t* created_ms, uint8_t* tombstones, uint64_t entries_cap,
                        uint64_t* n_out, int device);

/* The lazy rebuild of src/key_range/range.rs:117-128 (load_entries_from_file then
 * build_filter_from_entries): decode data.db on the filter's device and OR every key into its
 * bits (len_prefix = 1), no_of_elements += n.  *n_out (may be NULL) = entries decoded.
 * _dev: device data/blocks, queued on `stream` after one count readback.  _host: file bytes. */
int vbf_filter_rebuild_from_sst_dev(vbf_filter* f, const uint8_t* data, uint64_t len,
                                    const uint32_t* blocks, uint64_t nblocks, uint64_t* n_out,
                                    void* stream);
int vbf_filter_rebuild_from_sst_host(vbf_filter* f, const uint8_t* data, uint64_t len,
                                     const uint8_t* index, uint64_t index_len, uint64_t* n_out);

/* ---- batched read-path probe across SSTs ----
 * For n keys and nsst filters: out[j * nsst + s] = 1 iff SST s is a candidate for key j, i.e.
 * the key lies in [smallest_s, biggest_s] (Vec<u8> order; skipped when bounds_off is NULL) and
 * filters[s]->contains(key) -- the test KeyRange::filter_sstables_by_key_range applies per key
 * (src/key_range/range.rs:118,136).  Each key is hashed once for all filters.
 * filters: host array of handles, all on one device.  bounds / bounds_off (host): smallest_s =
 * bounds[bounds_off[2s] .. bounds_off[2s+1]), biggest_s = bounds[bounds_off[2s+1] ..
 * bounds_off[2s+2]).  A key reaching a filter with m == 0 and k > 0 is VBF_EDIVZERO (bf.rs:100):
 * without bounds every key reaches every filter, with bounds only the keys inside that SST's
 * range do (one extra readback when such a filter is present).  Host-resident filters are
 * rejected (vbf_filter_migrate them to the device first).
 * _dev: keys / offsets / out on that device, queued on `stream`.  _host: host buffers, synchronous. */
int vbf_multi_probe_dev(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                        int len_prefix, uint32_t nsst, const vbf_filter* const* filters,
                        const uint8_t* bounds, const uint64_t* bounds_off, uint8_t* out, void* stream);
int vbf_multi_probe_host(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                         int len_prefix, uint32_t nsst, const vbf_filter* const* filters,
                         const uint8_t* bounds, const uint64_t* bounds_off, uint8_t* out);
/* vbf_multi_probe_host's path for filters on several GPUs, with the split given: group[i] names
 * filter i's group, each group is probed on its first filter's device (all of a group's filters
 * must share it) and its answer columns are scattered back.  vbf_multi_probe_host calls it with
 * group[i] = the filter's device; a one-GPU host can exercise the split with any grouping. */
int vbf_multi_probe_host_grouped(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                                 int len_prefix, uint32_t nsst, const vbf_filter* const* filters,
                                 const uint8_t* bounds, const uint64_t* bounds_off, const int* group,
                                 uint8_t* out);

/* ---- compaction merge ----
 * One bucket of SizedTierRunner::merge_ssts_in_buckets (src/compactors/sized.rs:170-200): the
 * pairwise fold merged = tables[0], merged = merge_sstables(merged, t) (:207-283) with
 * tombstone_check (:286-320) at every pairwise merge.  Input: an arena of all tables' entries,
 * table r = entries run_off[r] .. run_off[r+1] (host array, run_off[0] = 0), each table strictly
 * increasing by key (a SkipMap; VBF_EINVAL otherwise); entry e = keys[offsets[e] ..
 * offsets[e+1]), created_ms[e] (i64 ms), tombstones[e] (0/1).  The compactor's tombstone map
 * enters as sorted unique keys (map_keys/map_off, map_n + 1 offsets) with times map_time;
 * map_n = 0 for an empty map.  TTLs as Config (use_ttl, entry_ttl, tombstone_ttl in ms) and
 * `now_ms` for Entry::has_expired (memtable/mem.rs:149-153: now > created + ttl).
 * Output: the merged table's entry ids in key order (out_ids, capacity = all entries), *n_out;
 * and, when upd_ids/upd_time are non-NULL, the keys whose map value changed (an entry id holding
 * the key) with their new time, *n_upd (capacity = all entries).  Synchronous on the stream. */
int vbf_compact_merge_dev(const uint8_t* keys, const uint64_t* offsets, const int64_t* created_ms,
                          const uint8_t* tombstones, const uint64_t* run_off, uint32_t nruns,
                          const uint8_t* map_keys, const uint64_t* map_off, const int64_t* map_time,
                          uint64_t map_n, int use_ttl, uint64_t entry_ttl_ms, uint64_t tombstone_ttl_ms,
                          uint64_t now_ms, uint32_t* out_ids, uint64_t* n_out, uint32_t* upd_ids,
                          int64_t* upd_time, uint64_t* n_upd, void* stream);
/* Same with every array in host memory, merged on `device`. */
int vbf_compact_merge_host(const uint8_t* keys, const uint64_t* offsets, const int64_t* created_ms,
                           const uint8_t* tombstones, const uint64_t* run_off, uint32_t nruns,
                           const uint8_t* map_keys, const uint64_t* map_off, const int64_t* map_time,
                           uint64_t map_n, int use_ttl, uint64_t entry_ttl_ms,
                           uint64_t tombstone_ttl_ms, uint64_t now_ms, uint32_t* out_ids,
                           uint64_t* n_out, uint32_t* upd_ids, int64_t* upd_time, uint64_t* n_upd,
                           int device);
/* ids -> the build's key layout: out_keys packed (capacity out_keys_cap), out_offsets n+1 (from 0),
 * and optionally the per-entry arrays (each needs its input).  *key_bytes (may be NULL) = packed
 * size.  Device pointers; one readback of the size. */
int vbf_gather_entries_dev(const uint8_t* keys, const uint64_t* offsets, const int64_t* created_ms,
                           const uint8_t* tombstones, const uint32_t* val_offsets, const uint32_t* ids,
                           uint64_t n, uint8_t* out_keys, uint64_t out_keys_cap, uint64_t* out_offsets,
                           int64_t* out_created_ms, uint8_t* out_tombstones, uint32_t* out_val_offsets,
                           uint64_t* key_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VBF_H */
