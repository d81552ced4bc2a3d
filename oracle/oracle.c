/*
 * oracle.c -- CPU restatement of velarixdb src/filter (TEST INFRASTRUCTURE ONLY; see oracle.h).
 *
 * Parity anchors (reference = /root/reference, velarixdb 0.0.17):
 *   calculate_hash                bf.rs:222-227   -> ora_hash
 *   calculate_no_of_bits          bf.rs:230-233   -> ora_num_bits
 *   calculate_no_of_hash_function bf.rs:236-239   -> ora_num_hash
 *   set / build_filter_from_entries bf.rs:84-92, :126-128 -> ora_build
 *   contains                      bf.rs:95-105    -> ora_probe, ora_probe_mt
 * Third-party algorithms restated from their published definitions (not in the reference tree):
 *   Rust std DefaultHasher = SipHash-1-3, keys (0,0) (Aumasson & Bernstein, "SipHash: a fast
 *     short-input PRF", c=1 compression / d=3 finalization rounds as used by Rust std);
 *     `Hash for [u8]` = write_usize(len) (8 bytes LE on x86-64) then write(bytes);
 *     `write_u64(seed)` appends LE64(seed) to the same stream.
 *   bit-vec 0.6.3 BitVec<u32>: set(i) = storage[i / 32] |= 1 << (i % 32).
 * Pinned by tests/golden/ (Perl-header SipHash vectors + reference SST fixtures).
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define ROTL(x, b) (uint64_t)(((x) << (b)) | ((x) >> (64 - (b))))
#define SIPROUND                                                                                   \
    do {                                                                                           \
        v0 += v1; v1 = ROTL(v1, 13); v1 ^= v0; v0 = ROTL(v0, 32);                                 \
        v2 += v3; v3 = ROTL(v3, 16); v3 ^= v2;                                                     \
        v0 += v3; v3 = ROTL(v3, 21); v3 ^= v0;                                                     \
        v2 += v1; v1 = ROTL(v1, 17); v1 ^= v2; v2 = ROTL(v2, 32);                                  \
    } while (0)

static uint64_t load_le64(const uint8_t* p) {
    uint64_t v;
    memcpy(&v, p, 8); /* x86-64 is little-endian */
    return v;
}

/* Streaming SipHash-1-3 state, the shape of Rust's SipHasher13 (write / finish). */
typedef struct {
    uint64_t v0, v1, v2, v3;
    uint64_t tail;   /* pending bytes, little-endian */
    unsigned ntail;  /* 0..7 */
    uint64_t length; /* total bytes written */
} sip13;

static void sip_init(sip13* s) {
    s->v0 = 0x736f6d6570736575ULL; /* k0 = 0 */
    s->v1 = 0x646f72616e646f6dULL; /* k1 = 0 */
    s->v2 = 0x6c7967656e657261ULL;
    s->v3 = 0x7465646279746573ULL;
    s->tail = 0;
    s->ntail = 0;
    s->length = 0;
}

static void sip_compress(sip13* s, uint64_t m) {
    uint64_t v0 = s->v0, v1 = s->v1, v2 = s->v2, v3 = s->v3;
    v3 ^= m;
    SIPROUND;
    v0 ^= m;
    s->v0 = v0; s->v1 = v1; s->v2 = v2; s->v3 = v3;
}

/* Byte-stream semantics; whole 8-byte words go straight to the compression function once
 * the pending tail is empty (the same bulk path Rust's SipHasher13::write takes). */
static void sip_write(sip13* s, const uint8_t* p, size_t len) {
    s->length += len;
    size_t i = 0;
    while (i < len && s->ntail != 0) {
        s->tail |= (uint64_t)p[i++] << (8 * s->ntail);
        if (++s->ntail == 8) {
            sip_compress(s, s->tail);
            s->tail = 0;
            s->ntail = 0;
        }
    }
    for (; i + 8 <= len; i += 8) sip_compress(s, load_le64(p + i));
    for (; i < len; ++i) s->tail |= (uint64_t)p[i] << (8 * s->ntail++);
}

static uint64_t sip_finish(const sip13* s) {
    uint64_t v0 = s->v0, v1 = s->v1, v2 = s->v2, v3 = s->v3;
    uint64_t b = ((s->length & 0xff) << 56) | s->tail;
    v3 ^= b;
    SIPROUND;
    v0 ^= b;
    v2 ^= 0xff;
    SIPROUND;
    SIPROUND;
    SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

uint64_t ora_siphash13(const uint8_t* msg, size_t len) {
    sip13 s;
    sip_init(&s);
    sip_write(&s, msg, len);
    return sip_finish(&s);
}

static void write_u64(sip13* s, uint64_t v) {
    uint8_t b[8];
    for (int i = 0; i < 8; ++i) b[i] = (uint8_t)(v >> (8 * i));
    sip_write(s, b, 8);
}

/* bf.rs:222-227: DefaultHasher::new(); key.hash(&mut h); h.write_u64(seed); h.finish() */
uint64_t ora_hash(const uint8_t* key, size_t len, int len_prefix, uint64_t seed) {
    sip13 s;
    sip_init(&s);
    if (len_prefix) write_u64(&s, (uint64_t)len); /* Hash for [u8]: write_length_prefix */
    sip_write(&s, key, len);
    write_u64(&s, seed);
    return sip_finish(&s);
}

/* Rust `f64 as u32`: saturating, NaN -> 0, truncation toward zero. */
static uint32_t f64_as_u32(double x) {
    if (x != x) return 0;
    if (x <= 0.0) return 0;
    if (x >= 4294967295.0) return 4294967295u;
    return (uint32_t)x;
}

/* bf.rs:230-233: -((n as f64 * p.ln()) / (2f64.ln()).powi(2)).ceil() as u32 */
uint32_t ora_num_bits(uint64_t n, double p) {
    const double ln2 = log(2.0);
    double x = ((double)n * log(p)) / (ln2 * ln2);
    return f64_as_u32(-ceil(x));
}

/* bf.rs:236-239: ((m as f64 / n as f64) * (2f64.ln()).ceil()) as u32 ; ln2.ceil() == 1.0 */
uint32_t ora_num_hash(uint32_t m, uint32_t n) {
    double x = ((double)m / (double)n) * ceil(log(2.0));
    return f64_as_u32(x);
}

static inline const uint8_t* key_at(const uint8_t* keys, const uint64_t* offsets, uint64_t stride,
                                    uint64_t j, uint64_t* len) {
    if (offsets) {
        *len = offsets[j + 1] - offsets[j];
        return keys + offsets[j];
    }
    *len = stride;
    return keys + j * stride;
}

int ora_build(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
              int len_prefix, uint32_t m, uint32_t k, uint32_t* words) {
    if (m == 0 && k > 0 && n > 0) return -1;
    for (uint64_t j = 0; j < n; ++j) {           /* bf.rs:127 entries.iter().for_each(set) */
        uint64_t len;
        const uint8_t* key = key_at(keys, offsets, stride, j, &len);
        for (uint32_t i = 0; i < k; ++i) {         /* bf.rs:86 */
            uint64_t h = ora_hash(key, len, len_prefix, i);
            uint64_t idx = h % (uint64_t)m;           /* bf.rs:88 */
            words[idx >> 5] |= 1u << (idx & 31);     /* bf.rs:89, bit-vec LSB-first u32 */
        }
    }
    return 0;
}

int ora_probe(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
              int len_prefix, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out) {
    if (m == 0 && k > 0 && n > 0) return -1;
    for (uint64_t j = 0; j < n; ++j) {
        uint64_t len;
        const uint8_t* key = key_at(keys, offsets, stride, j, &len);
        uint8_t hit = 1;                           /* bf.rs:104: vacuously true when k == 0 */
        for (uint32_t i = 0; i < k; ++i) {
            uint64_t idx = ora_hash(key, len, len_prefix, i) % (uint64_t)m;
            if (!((words[idx >> 5] >> (idx & 31)) & 1u)) { hit = 0; break; } /* bf.rs:100-102 */
        }
        out[j] = hit;
    }
    return 0;
}

void ora_hashes(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                int len_prefix, uint32_t k, uint64_t* out) {
    for (uint64_t j = 0; j < n; ++j) {
        uint64_t len;
        const uint8_t* key = key_at(keys, offsets, stride, j, &len);
        for (uint32_t i = 0; i < k; ++i) out[j * k + i] = ora_hash(key, len, len_prefix, i);
    }
}

/* ---- cpu-opt: prefix-shared hashing, threads OR private arrays together ---- */

typedef struct {
    const uint8_t* keys;
    const uint64_t* offsets;
    uint64_t stride, lo, hi;
    int len_prefix;
    uint32_t m, k;
    uint32_t* words;
} mt_job;

static void* mt_worker(void* arg) {
    mt_job* jb = (mt_job*)arg;
    for (uint64_t j = jb->lo; j < jb->hi; ++j) {
        uint64_t len;
        const uint8_t* key = key_at(jb->keys, jb->offsets, jb->stride, j, &len);
        sip13 pre;
        sip_init(&pre);
        if (jb->len_prefix) write_u64(&pre, len);
        sip_write(&pre, key, len);
        for (uint32_t i = 0; i < jb->k; ++i) {
            sip13 s = pre;
            write_u64(&s, i);
            uint64_t idx = sip_finish(&s) % (uint64_t)jb->m;
            jb->words[idx >> 5] |= 1u << (idx & 31);
        }
    }
    return NULL;
}

/* ORs the private arrays of threads 1.. into words[], each merging thread taking a word range
 * (the 2^32-bit config-5 filter is 512 MiB per thread: a serial merge of 16 took longer than the
 * hashing). */
typedef struct {
    uint32_t* words;
    mt_job* jobs;
    int threads;
    uint64_t lo, hi;
} mt_merge;

static void* mt_merger(void* arg) {
    mt_merge* mg = (mt_merge*)arg;
    for (int t = 1; t < mg->threads; ++t) {
        const uint32_t* src = mg->jobs[t].words;
        for (uint64_t w = mg->lo; w < mg->hi; ++w) mg->words[w] |= src[w];
    }
    return NULL;
}

int ora_build_mt(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                 int len_prefix, uint32_t m, uint32_t k, uint32_t* words, int threads) {
    if (m == 0 && k > 0 && n > 0) return -1;
    if (threads < 1) threads = 1;
    uint64_t nwords = ((uint64_t)m + 31) / 32;
    pthread_t* tid = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    mt_job* jobs = (mt_job*)calloc((size_t)threads, sizeof(mt_job));
    mt_merge* mg = (mt_merge*)calloc((size_t)threads, sizeof(mt_merge));
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (mt_job){keys, offsets, stride, n * t / threads, n * (t + 1) / threads,
                           len_prefix, m, k, NULL};
        jobs[t].words = t == 0 ? words : (uint32_t*)calloc(nwords ? nwords : 1, 4);
        pthread_create(&tid[t], NULL, mt_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    for (int t = 0; t < threads; ++t) {
        mg[t] = (mt_merge){words, jobs, threads, nwords * t / threads, nwords * (t + 1) / threads};
        pthread_create(&tid[t], NULL, mt_merger, &mg[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    for (int t = 1; t < threads; ++t) free(jobs[t].words);
    free(mg);
    free(jobs);
    free(tid);
    return 0;
}

/* contains (bf.rs:95-105) over key ranges on `threads` threads: the same answers as ora_probe
 * (each key's early-exit loop is unchanged; keys are independent). */
typedef struct {
    const uint8_t* keys;
    const uint64_t* offsets;
    uint64_t stride, lo, hi;
    int len_prefix;
    uint32_t m, k;
    const uint32_t* words;
    uint8_t* out;
} mt_probe_job;

static void* mt_prober(void* arg) {
    mt_probe_job* jb = (mt_probe_job*)arg;
    for (uint64_t j = jb->lo; j < jb->hi; ++j) {
        uint64_t len;
        const uint8_t* key = key_at(jb->keys, jb->offsets, jb->stride, j, &len);
        sip13 pre;
        sip_init(&pre);
        if (jb->len_prefix) write_u64(&pre, len);
        sip_write(&pre, key, len);
        uint8_t hit = 1;
        for (uint32_t i = 0; i < jb->k; ++i) {
            sip13 s = pre;
            write_u64(&s, i);
            uint64_t idx = sip_finish(&s) % (uint64_t)jb->m;
            if (!((jb->words[idx >> 5] >> (idx & 31)) & 1u)) { hit = 0; break; }
        }
        jb->out[j] = hit;
    }
    return NULL;
}

int ora_probe_mt(const uint8_t* keys, const uint64_t* offsets, uint64_t stride, uint64_t n,
                 int len_prefix, uint32_t m, uint32_t k, const uint32_t* words, uint8_t* out,
                 int threads) {
    if (m == 0 && k > 0 && n > 0) return -1;
    if (threads < 1) threads = 1;
    pthread_t* tid = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    mt_probe_job* jobs = (mt_probe_job*)calloc((size_t)threads, sizeof(mt_probe_job));
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (mt_probe_job){keys, offsets, stride, n * t / threads, n * (t + 1) / threads,
                                 len_prefix, m, k, words, out};
        pthread_create(&tid[t], NULL, mt_prober, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    free(jobs);
    free(tid);
    return 0;
}

/* ---- synthetic workloads ---- */

uint64_t ora_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

#define GOLDEN 0x9E3779B97F4A7C15ULL

static uint64_t fixed_word(uint64_t seed, uint64_t j, uint64_t c) {
    if (c == 0) return ora_splitmix64(seed ^ j);
    if (c == 1) return j;
    return ora_splitmix64(seed ^ j ^ (c * GOLDEN));
}

void ora_gen_fixed(uint64_t seed, uint64_t base, uint64_t n, uint32_t len, uint8_t* out) {
    for (uint64_t jj = 0; jj < n; ++jj) {
        uint64_t j = base + jj;
        uint8_t* o = out + jj * len;
        for (uint32_t b = 0; b < len; ++b) o[b] = (uint8_t)(fixed_word(seed, j, b >> 3) >> (8 * (b & 7)));
    }
}

/* Zipf(s = 1.1) on {1..121}: thresholds T[r] = floor(CDF(r) * 2^53), r = 1..120. */
static uint64_t zipf_T[121];
static int zipf_ready = 0;

static void zipf_init(void) {
    double w[122], total = 0.0;
    for (int r = 1; r <= 121; ++r) { w[r] = pow((double)r, -1.1); total += w[r]; }
    double acc = 0.0;
    for (int r = 1; r <= 120; ++r) {
        acc += w[r];
        zipf_T[r] = (uint64_t)((acc / total) * 9007199254740992.0);
    }
    zipf_ready = 1;
}

uint32_t ora_gen_var_len(uint64_t seed, uint64_t j) {
    if (!zipf_ready) zipf_init();
    uint64_t u = ora_splitmix64(seed ^ j ^ 0xD1B54A32D192ED03ULL) >> 11;
    uint32_t r = 1;
    while (r <= 120 && u >= zipf_T[r]) ++r;
    return 7 + r; /* 8..128 bytes */
}

/* Var key bytes: word 0 = (j << 8) | tag (tag = seed & 0xff), word c >= 1 = splitmix64(seed ^ j ^ c*GOLDEN). */
void ora_gen_var(uint64_t seed, uint64_t base, uint64_t n, const uint64_t* offsets, uint8_t* out) {
    for (uint64_t jj = 0; jj < n; ++jj) {
        uint64_t j = base + jj;
        uint64_t len = offsets[jj + 1] - offsets[jj];
        uint8_t* o = out + offsets[jj];
        for (uint64_t b = 0; b < len; ++b) {
            uint64_t c = b >> 3;
            uint64_t wv = c == 0 ? ((j << 8) | (seed & 0xff)) : ora_splitmix64(seed ^ j ^ (c * GOLDEN));
            o[b] = (uint8_t)(wv >> (8 * (b & 7)));
        }
    }
}

/* ---------------------------------------------------------------------------------------------
 * SST data.db / index.db: the step before the build on the recovery path.
 * ------------------------------------------------------------------------------------------- */

#define SST_BLOCK_SIZE 4096u /* consts/mod.rs:107 */
#define SST_ENTRY_FIXED 17u  /* u32 key_len + u32 value offset + u64 created_at + u8 tombstone */

static void put_le(uint8_t* p, uint64_t v, int nbytes) {
    for (int i = 0; i < nbytes; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
static uint64_t get_le(const uint8_t* p, int nbytes) {
    uint64_t v = 0;
    for (int i = 0; i < nbytes; ++i) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

/* Table::write_to_file (sst/table.rs:280-324) with Block::set_entry / is_full
 * (block/block_manager.rs:112-139: a block takes an entry unless size + (L + 17) > 4096, so an
 * entry over 4096 bytes fails the flush), Block::serialize (:168-190: u32 key_len | key |
 * u32 value offset | i64 created_at ms | u8 tombstone), write_block (table.rs:331-338: one index
 * entry per block = its LAST key and the block's start offset) and Index::serialize_entry
 * (index/indexer.rs:151-170: u32 key_len | key | u32 block offset).
 * data / index may be NULL to size the files.  Returns 0, or -1 when an entry exceeds a block. */
int ora_sst_write(const uint8_t* keys, const uint64_t* offsets, uint64_t n, const uint32_t* val_off,
                  const uint64_t* created_ms, const uint8_t* tomb, uint8_t* data, uint64_t* data_len,
                  uint8_t* index, uint64_t* index_len) {
    uint64_t dpos = 0, ipos = 0, blk_start = 0, blk_size = 0;
    int64_t last = -1; /* last entry of the open block */
    for (uint64_t j = 0; j <= n; ++j) {
        uint64_t es = 0;
        if (j < n) {
            es = (offsets[j + 1] - offsets[j]) + SST_ENTRY_FIXED;
            if (es > SST_BLOCK_SIZE) return -1;
        }
        if (last >= 0 && (j == n || blk_size + es > SST_BLOCK_SIZE)) { /* close the block */
            uint64_t L = offsets[last + 1] - offsets[last];
            if (index) {
                put_le(index + ipos, L, 4);
                memcpy(index + ipos + 4, keys + offsets[last], L);
                put_le(index + ipos + 4 + L, blk_start, 4);
            }
            ipos += L + 8;
            blk_start = dpos;
            blk_size = 0;
            last = -1;
        }
        if (j == n) break;
        uint64_t L = es - SST_ENTRY_FIXED;
        if (data) {
            put_le(data + dpos, L, 4);
            memcpy(data + dpos + 4, keys + offsets[j], L);
            put_le(data + dpos + 4 + L, val_off ? val_off[j] : 0, 4);
            put_le(data + dpos + 8 + L, created_ms ? created_ms[j] : 0, 8);
            data[dpos + 16 + L] = tomb ? (tomb[j] != 0) : 0;
        }
        dpos += es;
        blk_size += es;
        last = (int64_t)j;
    }
    *data_len = dpos;
    *index_len = ipos;
    return 0;
}

/* DataFileNode::load_entries (fs/mod.rs:275-332): sequential entries until EOF.  Output arrays
 * may be NULL (count only); offsets gets n+1 entries (absolute positions in keys).  tomb[j] =
 * (byte == 1) as the reference reads it.  Returns the entry count, or -1 on a truncated entry
 * (the reference's UnexpectedEof). */
int64_t ora_sst_decode(const uint8_t* data, uint64_t len, uint8_t* keys, uint64_t* offsets,
                       uint32_t* val_off, uint64_t* created_ms, uint8_t* tomb) {
    uint64_t p = 0, kb = 0;
    int64_t n = 0;
    while (p < len) {
        if (len - p < 4) return -1;
        uint64_t L = get_le(data + p, 4);
        if (len - p - 4 < L + 13) return -1;
        if (keys) memcpy(keys + kb, data + p + 4, L);
        if (offsets) offsets[n] = kb;
        if (val_off) val_off[n] = (uint32_t)get_le(data + p + 4 + L, 4);
        if (created_ms) created_ms[n] = get_le(data + p + 8 + L, 8);
        if (tomb) tomb[n] = data[p + 16 + L] == 1;
        kb += L;
        p += L + SST_ENTRY_FIXED;
        ++n;
    }
    if (offsets) offsets[n] = kb;
    return n;
}

/* index.db (indexer.rs:151-170) -> block start offsets.  offs may be NULL (count only).
 * Returns the block count, or -1 on a truncated entry. */
int64_t ora_sst_index_blocks(const uint8_t* index, uint64_t len, uint32_t* offs) {
    uint64_t p = 0;
    int64_t nb = 0;
    while (p < len) {
        if (len - p < 4) return -1;
        uint64_t L = get_le(index + p, 4);
        if (len - p - 4 < L + 4) return -1;
        if (offs) offs[nb] = (uint32_t)get_le(index + p + 4 + L, 4);
        p += L + 8;
        ++nb;
    }
    return nb;
}

/* ---------------------------------------------------------------------------------------------
 * Compaction merge: SizedTierRunner::merge_ssts_in_buckets folds a
 * bucket's tables pairwise -- merged = tables[0]; merged = merge_sstables(merged, t) for the
 * rest (compactors/sized.rs:170-200) -- and every pairwise merge passes each surviving entry
 * through tombstone_check (:286-320), whose `tombstones` map lives across merges and buckets
 * (cleared only when compaction finds nothing left to do, :73-75).  Restated literally here.
 * ------------------------------------------------------------------------------------------- */

typedef struct {
    uint8_t** keys;
    uint64_t* lens;
    int64_t* times;
    uint8_t* used;
    uint64_t cap, size;
} ora_tmap;

static uint64_t fnv(const uint8_t* k, uint64_t n) {
    uint64_t h = 1469598103934665603ULL;
    for (uint64_t i = 0; i < n; ++i) h = (h ^ k[i]) * 1099511628211ULL;
    return h;
}

void* ora_tmap_new(void) {
    ora_tmap* m = (ora_tmap*)calloc(1, sizeof(ora_tmap));
    m->cap = 1024;
    m->keys = (uint8_t**)calloc(m->cap, sizeof(uint8_t*));
    m->lens = (uint64_t*)calloc(m->cap, sizeof(uint64_t));
    m->times = (int64_t*)calloc(m->cap, sizeof(int64_t));
    m->used = (uint8_t*)calloc(m->cap, 1);
    return m;
}

void ora_tmap_free(void* p) {
    ora_tmap* m = (ora_tmap*)p;
    if (!m) return;
    for (uint64_t i = 0; i < m->cap; ++i) free(m->keys[i]);
    free(m->keys);
    free(m->lens);
    free(m->times);
    free(m->used);
    free(m);
}

static uint64_t tmap_slot(const ora_tmap* m, const uint8_t* k, uint64_t n) {
    uint64_t i = fnv(k, n) & (m->cap - 1);
    while (m->used[i] && !(m->lens[i] == n && (n == 0 || memcmp(m->keys[i], k, n) == 0))) i = (i + 1) & (m->cap - 1);
    return i;
}

int ora_tmap_get(void* p, const uint8_t* k, uint64_t n, int64_t* t) {
    ora_tmap* m = (ora_tmap*)p;
    uint64_t i = tmap_slot(m, k, n);
    if (!m->used[i]) return 0;
    *t = m->times[i];
    return 1;
}

void ora_tmap_set(void* p, const uint8_t* k, uint64_t n, int64_t t) {
    ora_tmap* m = (ora_tmap*)p;
    if (2 * (m->size + 1) > m->cap) { /* grow */
        ora_tmap old = *m;
        m->cap *= 2;
        m->keys = (uint8_t**)calloc(m->cap, sizeof(uint8_t*));
        m->lens = (uint64_t*)calloc(m->cap, sizeof(uint64_t));
        m->times = (int64_t*)calloc(m->cap, sizeof(int64_t));
        m->used = (uint8_t*)calloc(m->cap, 1);
        for (uint64_t i = 0; i < old.cap; ++i)
            if (old.used[i]) {
                uint64_t j = tmap_slot(m, old.keys[i], old.lens[i]);
                m->used[j] = 1;
                m->keys[j] = old.keys[i];
                m->lens[j] = old.lens[i];
                m->times[j] = old.times[i];
            }
        free(old.keys);
        free(old.lens);
        free(old.times);
        free(old.used);
    }
    uint64_t i = tmap_slot(m, k, n);
    if (!m->used[i]) {
        m->used[i] = 1;
        m->keys[i] = (uint8_t*)malloc(n ? n : 1);
        if (n) memcpy(m->keys[i], k, n);
        m->lens[i] = n;
        m->size++;
    }
    m->times[i] = t;
}

uint64_t ora_tmap_size(void* p) { return ((ora_tmap*)p)->size; }

/* Dump the map: keys into `keys` (NULL to size), lens, times; returns total key bytes. */
uint64_t ora_tmap_dump(void* p, uint8_t* keys, uint64_t* lens, int64_t* times) {
    ora_tmap* m = (ora_tmap*)p;
    uint64_t kb = 0, j = 0;
    for (uint64_t i = 0; i < m->cap; ++i)
        if (m->used[i]) {
            if (keys) memcpy(keys + kb, m->keys[i], m->lens[i]);
            if (lens) lens[j] = m->lens[i];
            if (times) times[j] = m->times[i];
            kb += m->lens[i];
            ++j;
        }
    return kb;
}

typedef struct {
    const uint8_t* keys;
    const uint64_t* offsets;
    const int64_t* created;
    const uint8_t* tomb;
    int use_ttl;
    uint64_t entry_ttl, tomb_ttl, now;
    ora_tmap* map;
} merge_ctx;

static int key_cmp(const merge_ctx* c, uint32_t a, uint32_t b) {
    const uint64_t la = c->offsets[a + 1] - c->offsets[a], lb = c->offsets[b + 1] - c->offsets[b];
    const uint64_t n = la < lb ? la : lb;
    int r = n ? memcmp(c->keys + c->offsets[a], c->keys + c->offsets[b], n) : 0;
    if (r) return r < 0 ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

/* Entry::has_expired (memtable/mem.rs:149-153): now > created + ttl, in u64 ms. */
static int expired(const merge_ctx* c, uint32_t e, uint64_t ttl) {
    return c->now > (uint64_t)c->created[e] + ttl;
}

/* tombstone_check (sized.rs:291-320). */
static void tomb_check(merge_ctx* c, uint32_t e, uint32_t* out, uint64_t* n_out) {
    const uint8_t* k = c->keys + c->offsets[e];
    const uint64_t n = c->offsets[e + 1] - c->offsets[e];
    int ins = 0;
    int64_t t;
    if (ora_tmap_get(c->map, k, n, &t)) {
        if (c->created[e] > t) {
            if (c->tomb[e]) {
                ora_tmap_set(c->map, k, n, c->created[e]);
                ins = !expired(c, e, c->tomb_ttl);
            } else if (c->use_ttl) {
                ins = !expired(c, e, c->entry_ttl);
            } else {
                ins = 1;
            }
        }
    } else if (c->tomb[e]) {
        ora_tmap_set(c->map, k, n, c->created[e]);
        ins = !expired(c, e, c->tomb_ttl);
    } else if (c->use_ttl) {
        ins = !expired(c, e, c->entry_ttl);
    } else {
        ins = 1;
    }
    if (ins) out[(*n_out)++] = e;
}

/* One bucket: entries of table t are ids run_off[t] .. run_off[t+1] (each table sorted by key,
 * unique -- a SkipMap).  Writes the merged table's entry ids in key order to out_ids and returns
 * their count; `tmap` carries the tombstone map in and out. */
int64_t ora_compact_merge(const uint8_t* keys, const uint64_t* offsets, const int64_t* created,
                          const uint8_t* tomb, const uint64_t* run_off, uint32_t nruns, int use_ttl,
                          uint64_t entry_ttl_ms, uint64_t tomb_ttl_ms, uint64_t now_ms, void* tmap,
                          uint32_t* out_ids) {
    merge_ctx c = {keys, offsets, created, tomb, use_ttl, entry_ttl_ms, tomb_ttl_ms, now_ms, (ora_tmap*)tmap};
    if (nruns == 0) return 0;
    const uint64_t total = run_off[nruns] - run_off[0];
    uint32_t* cur = (uint32_t*)malloc((total + 1) * sizeof(uint32_t));
    uint32_t* nxt = (uint32_t*)malloc((total + 1) * sizeof(uint32_t));
    uint64_t ncur = 0;
    for (uint64_t e = run_off[0]; e < run_off[1]; ++e) cur[ncur++] = (uint32_t)e; /* merged = tables[0] */
    for (uint32_t t = 1; t < nruns; ++t) {                                        /* merge_sstables */
        uint64_t p1 = 0, p2 = run_off[t], e2 = run_off[t + 1], nn = 0;
        while (p1 < ncur && p2 < e2) {
            const int r = key_cmp(&c, cur[p1], (uint32_t)p2);
            if (r < 0) {
                tomb_check(&c, cur[p1++], nxt, &nn);
            } else if (r == 0) {
                if (created[cur[p1]] > created[p2]) tomb_check(&c, cur[p1], nxt, &nn);
                else tomb_check(&c, (uint32_t)p2, nxt, &nn);
                ++p1;
                ++p2;
            } else {
                tomb_check(&c, (uint32_t)p2++, nxt, &nn);
            }
        }
        while (p1 < ncur) tomb_check(&c, cur[p1++], nxt, &nn);
        while (p2 < e2) tomb_check(&c, (uint32_t)p2++, nxt, &nn);
        uint32_t* sw = cur;
        cur = nxt;
        nxt = sw;
        ncur = nn;
    }
    memcpy(out_ids, cur, ncur * sizeof(uint32_t));
    free(cur);
    free(nxt);
    return (int64_t)ncur;
}
