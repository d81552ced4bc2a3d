/*
 * oracle.h -- CPU restatement of velarixdb's Bloom-filter path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the *checker*.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product (velarixdb_amd/libvbf.so) never links it and
 * never falls back to it.
 *
 * Reference: /root/reference/src/filter/bf.rs (velarixdb 0.0.17).  The arithmetic lives in
 * two third-party crates that are NOT vendored in the reference (no Cargo.lock):
 *   - Rust std `DefaultHasher` (toolchain "stable", unpinned) = SipHash-1-3 with k0 = k1 = 0;
 *   - `bit-vec` 0.6.3 (Cargo.toml:19): BitVec<u32>, bit i = word[i/32] bit (i%32), LSB first.
 * Parity is pinned by golden vectors from an independent SipHash implementation (the Perl
 * header shipped in this container) and by the reference's own fixtures (tests/golden/).
 */
#ifndef VELARIX_ORACLE_H
#define VELARIX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* SipHash-1-3, keys (0,0), over an arbitrary message. std DefaultHasher::new(). */
uint64_t ora_siphash13(const uint8_t* msg, size_t len);

/* calculate_hash (bf.rs:222-227): message = [LE64(len) if len_prefix] || key || LE64(seed). */
uint64_t ora_hash(const uint8_t* key, size_t len, int len_prefix, uint64_t seed);

/* calculate_no_of_bits (bf.rs:230-233), Rust `as u32` saturating cast included. */
uint32_t ora_num_bits(uint64_t n, double p);

/* calculate_no_of_hash_function (bf.rs:236-239). */
uint32_t ora_num_hash(uint32_t m, uint32_t n);

/* Key-set addressing: key j = keys[offsets[j] .. offsets[j+1]) when offsets != NULL,
 * otherwise keys[j*stride .. j*stride + stride). */

/* build_filter_from_entries -> set (bf.rs:126-128, :84-92), reference-faithful loop:
 * full SipHash per seed, u64 % m, OR into words.  Returns 0, or -1 when m == 0 && k > 0
 * (the reference panics: division by zero at bf.rs:88). */
int ora_build(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
              int len_prefix, uint32_t m, uint32_t k, uint32_t* words);

/* Same result, multi-threaded with prefix-shared hashing (the "cpu-opt" baseline). */
int ora_build_mt(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                 int len_prefix, uint32_t m, uint32_t k, uint32_t* words, int threads);

/* contains (bf.rs:95-105): early-exit probe, out[j] = 0/1. */
int ora_probe(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
              int len_prefix, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out);

/* The same answers on `threads` threads (keys split into ranges). */
int ora_probe_mt(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                 int len_prefix, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
                 int threads);

/* Raw hashes, out[j*k + i] = calculate_hash(key_j, i). */
void ora_hashes(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                int len_prefix, uint32_t k, uint64_t* out);

/* Synthetic workloads. */
uint64_t ora_splitmix64(uint64_t x);
/* Fixed-length keys: key_j = LE64(splitmix64(seed ^ (base+j))) || LE64(base+j) || ... for L>16
 * the tail continues with LE64(splitmix64(seed ^ (base+j) ^ (c * 0x9E37...))) words. */
void ora_gen_fixed(uint64_t seed, uint64_t base, uint64_t n, uint32_t len, uint8_t* out);
/* Variable-length keys, length 7 + r, r ~ Zipf(s) on {1..121}, see ora_gen_var_len. */
uint32_t ora_gen_var_len(uint64_t seed, uint64_t j);
void ora_gen_var(uint64_t seed, uint64_t base, uint64_t n, const uint64_t* offsets, uint8_t* out);


/* SST files, see oracle.c for the reference anchors:
 * writer (table.rs:280-338, block_manager.rs:112-190, indexer.rs:130-170), data.db decoder
 * (fs/mod.rs:275-332) and index.db -> block start offsets. */
int ora_sst_write(const uint8_t* keys, const uint64_t* offsets, uint64_t n, const uint32_t* val_off,
                  const uint64_t* created_ms, const uint8_t* tomb, uint8_t* data, uint64_t* data_len,
                  uint8_t* index, uint64_t* index_len);
int64_t ora_sst_decode(const uint8_t* data, uint64_t len, uint8_t* keys, uint64_t* offsets,
                       uint32_t* val_off, uint64_t* created_ms, uint8_t* tomb);
int64_t ora_sst_index_blocks(const uint8_t* index, uint64_t len, uint32_t* offs);

/* Compaction merge: the pairwise fold of compactors/sized.rs:170-283 with
 * tombstone_check (:286-320) and its persistent tombstone map (an opaque handle here). */
void* ora_tmap_new(void);
void ora_tmap_free(void* m);
void ora_tmap_set(void* m, const uint8_t* key, uint64_t len, int64_t t);
int ora_tmap_get(void* m, const uint8_t* key, uint64_t len, int64_t* t);
uint64_t ora_tmap_size(void* m);
uint64_t ora_tmap_dump(void* m, uint8_t* keys, uint64_t* lens, int64_t* times);
int64_t ora_compact_merge(const uint8_t* keys, const uint64_t* offsets, const int64_t* created,
                          const uint8_t* tomb, const uint64_t* run_off, uint32_t nruns, int use_ttl,
                          uint64_t entry_ttl_ms, uint64_t tomb_ttl_ms, uint64_t now_ms, void* tmap,
                          uint32_t* out_ids);

#ifdef __cplusplus
}
#endif
#endif
