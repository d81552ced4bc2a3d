/* c_host.c -- libvbf.so from a plain C host: no Python, no PyTorch, only include/vbf.h.
 *
 * This is the call sequence a Rust caller makes through FFI:
 * BloomFilter::new (bf.rs:62-81) -> build_filter_from_entries (bf.rs:126-128) -> contains
 * (bf.rs:95-105) -> serialize (bf.rs:158-172) -> the bit words (filter.db persistence), plus the
 * compaction fan-in's sharded builds (sized.rs:192-193 per merged table).
 *
 * usage: c_host KEYS_FILE N STRIDE P OUT_PREFIX
 *   KEYS_FILE : N keys of STRIDE bytes, back to back (hashed as Vec<u8>: len_prefix = 1)
 *   writes OUT_PREFIX.words (the filter's u32 words), OUT_PREFIX.meta (16-byte filter.db),
 *   OUT_PREFIX.shards (words of two shard builds: first half / second half of the keys, at the
 *   same m and k), OUT_PREFIX.filterdb (filter.db with the bit array persisted after the 16 bytes,
 *   vbf_filter_serialize_ext) and prints one line: "m k hits n restored async_equal".
 * The persisted file is read back (vbf_filter_recover_ext: restored = 1, same words, no rebuild),
 * and a second filter is built with vbf_filter_set_host_async from the caller's buffer (released
 * through the callback, as a Rust caller drops its packed Vec): async_equal = 1 when its words
 * equal the synchronous build's.
 * Exit status 0 on success; any library failure prints vbf_last_error() and exits 1. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vbf.h"

static void check(int rc, const char* what) {
    if (rc != VBF_OK) {
        fprintf(stderr, "%s failed (%d): %s\n", what, rc, vbf_last_error());
        exit(1);
    }
}

static int released = 0;
static void release_keys(void* ctx) { released += (ctx != NULL); }

static void write_file(const char* prefix, const char* ext, const void* p, size_t n) {
    char path[4096];
    snprintf(path, sizeof path, "%s.%s", prefix, ext);
    FILE* f = fopen(path, "wb");
    if (!f || fwrite(p, 1, n, f) != n) {
        fprintf(stderr, "cannot write %s\n", path);
        exit(1);
    }
    fclose(f);
}

int main(int argc, char** argv) {
    if (argc != 6) {
        fprintf(stderr, "usage: %s KEYS_FILE N STRIDE P OUT_PREFIX\n", argv[0]);
        return 2;
    }
    const uint64_t n = strtoull(argv[2], NULL, 10), stride = strtoull(argv[3], NULL, 10);
    const double p = strtod(argv[4], NULL);
    uint8_t* keys = malloc(n * stride + 1);
    FILE* kf = fopen(argv[1], "rb");
    if (!keys || !kf || fread(keys, 1, n * stride, kf) != n * stride) {
        fprintf(stderr, "cannot read %llu keys from %s\n", (unsigned long long)n, argv[1]);
        return 1;
    }
    fclose(kf);

    int ndev = 0;
    check(vbf_device_count(&ndev), "vbf_device_count");
    if (ndev < 1) {
        fprintf(stderr, "no gfx950 device\n");
        return 1;
    }

    vbf_filter* f = NULL;
    check(vbf_filter_new(p, n, 0, &f), "vbf_filter_new");
    check(vbf_filter_set_host(f, keys, NULL, stride, n, 1), "vbf_filter_set_host");
    uint8_t* hit = malloc(n + 1);
    check(vbf_filter_contains_host(f, keys, NULL, stride, n, 1, hit), "vbf_filter_contains_host");
    uint64_t hits = 0;
    for (uint64_t j = 0; j < n; ++j) hits += hit[j];

    const uint32_t m = vbf_filter_num_bits(f), k = vbf_filter_num_hash_functions(f);
    const uint64_t nw = ((uint64_t)m + 31) / 32;
    uint32_t* words = calloc(nw + 1, 4);
    check(vbf_filter_words_to_host(f, words, nw), "vbf_filter_words_to_host");
    uint8_t meta[16];
    check(vbf_filter_serialize(f, meta), "vbf_filter_serialize");
    write_file(argv[5], "words", words, nw * 4);
    write_file(argv[5], "meta", meta, 16);

    /* two independent shard builds at the same m, k (one per merged table in a compaction) */
    uint32_t* sw = calloc(2 * nw + 1, 4);
    const uint64_t h = n / 2;
    vbf_shard sh[2] = {
        {keys, NULL, stride, h, 1, m, k, sw, nw, 0},
        {keys + h * stride, NULL, stride, n - h, 1, m, k, sw + nw, nw, 0},
    };
    const int devs[1] = {0};
    check(vbf_build_shards_host(sh, 2, devs, 1), "vbf_build_shards_host");
    write_file(argv[5], "shards", sw, 2 * nw * 4);

    /* filter.db with persisted bits (bf.rs:114-123 write + the extension), read back the way
     * the lazy recovery of range.rs:117-128 would, without the rebuild */
    uint64_t flen = 0;
    check(vbf_filter_serialize_ext(f, NULL, NULL, 0, n, 1, NULL, 0, &flen), "serialize_ext(size)");
    uint8_t* fdb = malloc(flen);
    check(vbf_filter_serialize_ext(f, NULL, NULL, 0, n, 1, fdb, flen, &flen), "serialize_ext");
    write_file(argv[5], "filterdb", fdb, flen);
    vbf_filter* r = NULL;
    int restored = 0;
    check(vbf_filter_recover_ext(fdb, flen, 0, &r, &restored), "recover_ext");
    uint32_t* rw = calloc(nw + 1, 4);
    check(vbf_filter_words_to_host(r, rw, nw), "words(recovered)");
    if (memcmp(rw, words, nw * 4) != 0 || vbf_filter_num_elements(r) != 2 * (uint32_t)n) restored = 0;

    /* the asynchronous build from the caller's buffer */
    vbf_filter* a = NULL;
    check(vbf_filter_new(p, n, VBF_DEVICE_AUTO, &a), "vbf_filter_new(auto)");
    check(vbf_filter_set_host_async(a, keys, NULL, stride, n, 1, release_keys, keys), "set_host_async");
    check(vbf_filter_sync(a), "vbf_filter_sync");
    check(vbf_filter_words_to_host(a, rw, nw), "words(async)");
    const int async_equal = released == 1 && memcmp(rw, words, nw * 4) == 0;

    printf("%u %u %llu %llu %d %d\n", m, k, (unsigned long long)hits, (unsigned long long)n, restored, async_equal);
    vbf_filter_free(r);
    vbf_filter_free(a);
    free(fdb);
    free(rw);
    vbf_filter_free(f);
    free(keys);
    free(hit);
    free(words);
    free(sw);
    return 0;
}
