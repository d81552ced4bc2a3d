/* rust_replay.c -- the call sequence of INTEGRATION.md's patched src/filter/bf.rs bodies, replayed
 * from plain C (no Rust toolchain in this image; no Python or PyTorch in this process).
 *
 * Each bf_* function below is one patched Rust method, making exactly the FFI calls its Rust body
 * makes, on a struct with the patched BloomFilter's fields -- all of them public, so velarixdb's
 * own `BloomFilter { file_path: Some(..), ..Default::default() }` (db/recovery.rs:143-146,
 * tests/workload.rs:309-312) keeps compiling:
 *
 *   pub struct BloomFilter { sst_dir, no_of_hash_func, handle: FilterHandle, false_positive_rate,
 *                            file_path }                                          (bf.rs:37-58)
 *
 * Scenarios (the reference's callers):
 *   1. compaction (compactors/sized.rs:192-193): new -> build_filter_from_entries -> write
 *   2. restart, persisted bits (db/recovery.rs:143-146 then key_range/range.rs:117-128):
 *      Default{file_path} -> recover_meta -> build_filter_from_entries (skipped) -> contains
 *   3. restart, memtable-born SST (a 16-byte filter.db, memtable/mem.rs:191,209-211 then flush):
 *      new (host) -> per-key contains + set -> write -> Default{file_path} -> recover_meta ->
 *      build_filter_from_entries (a GPU rebuild)
 *   4. Clone (bf.rs:242-254) of the recovered filter, then set on the clone: the clone's count
 *      diverges, the bits stay shared.
 *
 * usage: rust_replay KEYS OFFSETS N P DIR
 *   KEYS: the entries' key bytes back to back; OFFSETS: N + 1 u64 absolute offsets into KEYS
 *   (a SkipMap's keys as ffi::pack lays them out).  Writes DIR/sst1/filter.db, DIR/sst2/filter.db,
 *   DIR/{built,recovered,memtable,rebuilt}.words and prints one JSON line. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "vbf.h"

static void check(int rc, const char* what) { /* ffi::check(..).expect(..) */
    if (rc != VBF_OK) {
        fprintf(stderr, "%s failed (%d): %s\n", what, rc, vbf_last_error());
        exit(1);
    }
}

/* ---- FilterHandle: one owned *mut VbfFilter (Send + Sync, Clone, Default, Drop, Debug) ---- */
typedef struct {
    vbf_filter* raw;
} FilterHandle;

static FilterHandle handle_default(void) { /* impl Default: vbf_filter_default(VBF_DEVICE_HOST) */
    FilterHandle h = {NULL};
    check(vbf_filter_default(VBF_DEVICE_HOST, &h.raw), "vbf_filter_default");
    return h;
}
static FilterHandle handle_clone(const FilterHandle* h) { /* impl Clone: bits shared, count copied */
    FilterHandle c = {NULL};
    check(vbf_filter_clone(h->raw, &c.raw), "vbf_filter_clone");
    return c;
}
static void handle_drop(FilterHandle* h) { /* impl Drop */
    vbf_filter_free(h->raw);
    h->raw = NULL;
}

/* ---- the patched BloomFilter ---- */
typedef struct {
    char sst_dir[1024];
    size_t no_of_hash_func;
    FilterHandle handle;
    double false_positive_rate;
    char file_path[1200];
} BloomFilter;

/* impl Default (bf.rs:256-267) */
static BloomFilter bf_default(void) {
    BloomFilter f;
    memset(&f, 0, sizeof f);
    f.handle = handle_default();
    return f;
}

/* BloomFilter::new (bf.rs:62-81): host-resident (the memtable's filter; a compaction filter moves
 * to its GPU in build_filter_from_entries) */
static BloomFilter bf_new(double p, uint64_t n) {
    BloomFilter f;
    memset(&f, 0, sizeof f);
    check(vbf_filter_new(p, n, VBF_DEVICE_HOST, &f.handle.raw), "vbf_filter_new");
    f.no_of_hash_func = vbf_filter_num_hash_functions(f.handle.raw);
    f.false_positive_rate = p;
    return f;
}

/* impl Clone (bf.rs:242-254) */
static BloomFilter bf_clone(const BloomFilter* s) {
    BloomFilter c = *s;
    c.handle = handle_clone(&s->handle);
    return c;
}

/* ffi::message: the bytes `key.hash(&mut RecordingHasher)` writes for a Vec<u8> key */
static uint8_t* message(const uint8_t* key, uint64_t len, uint64_t* mlen) {
    uint8_t* m = malloc(len + 8);
    memcpy(m, &len, 8); /* write_usize(len), native-endian (x86-64: little) */
    memcpy(m + 8, key, len);
    *mlen = len + 8;
    return m;
}

/* set (bf.rs:84-92) */
static void bf_set(BloomFilter* f, const uint8_t* key, uint64_t len) {
    uint64_t ml;
    uint8_t* msg = message(key, len, &ml);
    const uint64_t offs[2] = {0, ml};
    check(vbf_filter_set_host(f->handle.raw, msg, offs, 0, 1, 0), "Bloom set failed");
    free(msg);
}

/* contains (bf.rs:95-105) */
static int bf_contains(const BloomFilter* f, const uint8_t* key, uint64_t len) {
    uint64_t ml;
    uint8_t* msg = message(key, len, &ml);
    const uint64_t offs[2] = {0, ml};
    uint8_t out = 0;
    check(vbf_filter_contains_host(f->handle.raw, msg, offs, 0, 1, 0, &out), "Bloom probe failed");
    free(msg);
    return out != 0;
}

/* the Box<(Vec<u8>, Vec<u64>)> handed to set_host_async; ffi::drop_packed frees it */
typedef struct {
    uint8_t* keys;
    uint64_t* offsets;
} Packed;
static int g_released = 0;
static void drop_packed(void* ctx) {
    Packed* p = ctx;
    free(p->keys);
    free(p->offsets);
    free(p);
    ++g_released;
}

/* build_filter_from_entries (bf.rs:126-128); returns 1 when the persisted bits made it a no-op */
static int bf_build_filter_from_entries(BloomFilter* f, const uint8_t* keys, const uint64_t* offsets,
                                        uint64_t n) {
    const int restored = vbf_filter_take_restored(f->handle.raw);
    check(restored < 0 ? restored : 0, "vbf_filter_take_restored");
    if (restored) return 1;
    check(vbf_filter_migrate(f->handle.raw, VBF_DEVICE_AUTO), "migrate failed");
    Packed* p = malloc(sizeof *p); /* ffi::pack(entries.iter().map(|e| e.key().as_slice())) */
    const uint64_t bytes = offsets[n] - offsets[0];
    p->keys = malloc(bytes + 1);
    p->offsets = malloc((n + 1) * 8);
    memcpy(p->keys, keys + offsets[0], bytes);
    for (uint64_t i = 0; i <= n; ++i) p->offsets[i] = offsets[i] - offsets[0];
    check(vbf_filter_set_host_async(f->handle.raw, p->keys, p->offsets, 0, n, 1, drop_packed, p),
          "GPU Bloom build failed");
    check(vbf_filter_set_sst_entries(f->handle.raw, n), "vbf_filter_set_sst_entries");
    return 0;
}

static void write_bytes(const char* path, const void* p, size_t n) {
    FILE* fp = fopen(path, "wb");
    if (!fp || fwrite(p, 1, n, fp) != n) {
        fprintf(stderr, "cannot write %s\n", path);
        exit(1);
    }
    fclose(fp);
}

/* write (bf.rs:114-123): the 16 bytes, then the bits when the filter knows its SST's entries */
static void bf_write(BloomFilter* f, const char* dir) {
    const uint64_t entries = vbf_filter_sst_entries(f->handle.raw);
    uint64_t len = 0;
    check(vbf_filter_serialize_ext(f->handle.raw, NULL, NULL, 0, entries, 1, NULL, 0, &len),
          "GPU Bloom build or size failed");
    uint8_t* buf = malloc(len);
    check(vbf_filter_serialize_ext(f->handle.raw, NULL, NULL, 0, entries, 1, buf, len, &len), "serialize");
    mkdir(dir, 0755);
    snprintf(f->file_path, sizeof f->file_path, "%s/filter.db", dir);
    write_bytes(f->file_path, buf, len);
    free(buf);
}

/* recover_meta (bf.rs:135-150) */
static void bf_recover_meta(BloomFilter* f) {
    FILE* fp = fopen(f->file_path, "rb");
    if (!fp) {
        fprintf(stderr, "FilterFileOpen %s\n", f->file_path);
        exit(1);
    }
    fseek(fp, 0, SEEK_END);
    const long len = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    uint8_t* bytes = malloc(len + 1);
    if (fread(bytes, 1, len, fp) != (size_t)len) exit(1);
    fclose(fp);
    vbf_filter* raw = NULL;
    int restored = 0;
    check(vbf_filter_recover_ext(bytes, len, VBF_DEVICE_AUTO, &raw, &restored), "recover");
    handle_drop(&f->handle); /* self.handle = FilterHandle(raw) */
    f->handle.raw = raw;
    f->no_of_hash_func = vbf_filter_num_hash_functions(raw);
    f->false_positive_rate = vbf_filter_false_positive_rate(raw);
    free(bytes);
}

static void dump_words(const BloomFilter* f, const char* dir, const char* name) {
    const uint64_t nw = ((uint64_t)vbf_filter_num_bits(f->handle.raw) + 31) / 32;
    uint32_t* w = calloc(nw + 1, 4);
    check(vbf_filter_words_to_host(f->handle.raw, w, nw), "words");
    char path[1200];
    snprintf(path, sizeof path, "%s/%s.words", dir, name);
    write_bytes(path, w, nw * 4);
    free(w);
}

static void* read_all(const char* path, size_t want) {
    FILE* fp = fopen(path, "rb");
    uint8_t* p = malloc(want + 1);
    if (!fp || fread(p, 1, want, fp) != want) {
        fprintf(stderr, "cannot read %zu bytes from %s\n", want, path);
        exit(1);
    }
    fclose(fp);
    return p;
}

int main(int argc, char** argv) {
    if (argc != 6) {
        fprintf(stderr, "usage: %s KEYS OFFSETS N P DIR\n", argv[0]);
        return 2;
    }
    const uint64_t n = strtoull(argv[3], NULL, 10);
    const double p = strtod(argv[4], NULL);
    const char* dir = argv[5];
    uint64_t* offsets = read_all(argv[2], (n + 1) * 8);
    uint8_t* keys = read_all(argv[1], offsets[n]);
    char d1[1100], d2[1100];
    snprintf(d1, sizeof d1, "%s/sst1", dir);
    snprintf(d2, sizeof d2, "%s/sst2", dir);

    /* 1. compaction: BloomFilter::new + build_filter_from_entries, then the SST's write */
    BloomFilter built = bf_new(p, n);
    const int skipped1 = bf_build_filter_from_entries(&built, keys, offsets, n);
    bf_write(&built, d1); /* waits for the queued GPU build */
    dump_words(&built, dir, "built");

    /* 2. restart: the stub of db/recovery.rs:143-146, then the lazy rebuild of range.rs:117-128 */
    BloomFilter rec = bf_default();
    snprintf(rec.file_path, sizeof rec.file_path, "%s/filter.db", d1);
    bf_recover_meta(&rec);
    const int skipped2 = bf_build_filter_from_entries(&rec, keys, offsets, n);
    uint64_t hits = 0;
    for (uint64_t j = 0; j < n; ++j) hits += bf_contains(&rec, keys + offsets[j], offsets[j + 1] - offsets[j]);
    dump_words(&rec, dir, "recovered");

    /* 3. a memtable-born SST: per-key contains + set (mem.rs:209-211) into a filter sized for half
     * the keys, flushed with its 16 bytes only, recovered at m = num_bits(stored n, p) and rebuilt */
    BloomFilter mt = bf_new(p, n / 2);
    for (uint64_t j = 0; j < n; ++j) {
        const uint8_t* kp = keys + offsets[j];
        const uint64_t kl = offsets[j + 1] - offsets[j];
        if (!bf_contains(&mt, kp, kl)) bf_set(&mt, kp, kl);
    }
    const uint32_t mt_n = vbf_filter_num_elements(mt.handle.raw);
    dump_words(&mt, dir, "memtable");
    bf_write(&mt, d2);
    BloomFilter rb = bf_default();
    snprintf(rb.file_path, sizeof rb.file_path, "%s/filter.db", d2);
    bf_recover_meta(&rb);
    const int skipped3 = bf_build_filter_from_entries(&rb, keys, offsets, n);
    uint64_t rb_hits = 0;
    for (uint64_t j = 0; j < n; ++j) rb_hits += bf_contains(&rb, keys + offsets[j], offsets[j + 1] - offsets[j]);
    dump_words(&rb, dir, "rebuilt");

    /* 4. Clone, then set on the clone: count copied (diverges), bits shared */
    BloomFilter c = bf_clone(&rec);
    const uint32_t n_before = vbf_filter_num_elements(rec.handle.raw);
    const uint8_t fresh[] = "a key set only through the clone";
    const int fresh_before = bf_contains(&rec, fresh, sizeof fresh - 1);
    bf_set(&c, fresh, sizeof fresh - 1);
    const int fresh_in_orig = bf_contains(&rec, fresh, sizeof fresh - 1);
    const uint32_t n_orig = vbf_filter_num_elements(rec.handle.raw), n_clone = vbf_filter_num_elements(c.handle.raw);
    const uint64_t nw = ((uint64_t)vbf_filter_num_bits(rec.handle.raw) + 31) / 32;
    uint32_t* wa = calloc(nw + 1, 4);
    uint32_t* wb = calloc(nw + 1, 4);
    check(vbf_filter_words_to_host(rec.handle.raw, wa, nw), "words(orig)");
    check(vbf_filter_words_to_host(c.handle.raw, wb, nw), "words(clone)");
    const int shared = memcmp(wa, wb, nw * 4) == 0;
    dump_words(&c, dir, "cloned");

    /* Default's fields as FRU leaves them: m = 0, k = 0, n = 0, host-resident (BitVec::new()) */
    BloomFilter d = bf_default();
    const int default_ok = vbf_filter_num_bits(d.handle.raw) == 0 && vbf_filter_num_hash_functions(d.handle.raw) == 0 &&
                           vbf_filter_num_elements(d.handle.raw) == 0 && vbf_filter_device(d.handle.raw) == VBF_DEVICE_HOST &&
                           d.no_of_hash_func == 0 && d.false_positive_rate == 0.0 && d.sst_dir[0] == 0;

    printf("{\"m\": %u, \"k\": %u, \"rec_m\": %u, \"rec_k\": %zu, \"rec_n\": %u, \"skipped\": [%d, %d, %d], "
           "\"hits\": %llu, \"mt_m\": %u, \"mt_n\": %u, \"rb_m\": %u, \"rb_n\": %u, \"rb_hits\": %llu, "
           "\"released\": %d, \"n_before\": %u, \"n_orig\": %u, \"n_clone\": %u, \"fresh_before\": %d, "
           "\"fresh_in_orig\": %d, \"shared\": %d, \"default_ok\": %d, \"rec_device\": %d}\n",
           vbf_filter_num_bits(built.handle.raw), vbf_filter_num_hash_functions(built.handle.raw),
           vbf_filter_num_bits(rec.handle.raw), rec.no_of_hash_func, n_before,
           skipped1, skipped2, skipped3, (unsigned long long)hits, vbf_filter_num_bits(mt.handle.raw), mt_n,
           vbf_filter_num_bits(rb.handle.raw), vbf_filter_num_elements(rb.handle.raw), (unsigned long long)rb_hits,
           g_released, n_before, n_orig, n_clone, fresh_before, fresh_in_orig, shared, default_ok,
           vbf_filter_device(rec.handle.raw));
    handle_drop(&c.handle);
    handle_drop(&d.handle);
    handle_drop(&rb.handle);
    handle_drop(&mt.handle);
    handle_drop(&rec.handle);
    handle_drop(&built.handle);
    free(wa);
    free(wb);
    free(keys);
    free(offsets);
    return 0;
}
