/* memtable_latency.c -- single-key latency of the memtable's filter calls, from a plain C host.
 *
 * velarixdb's memtable calls contains then set on every put (src/memtable/mem.rs:209-211) and
 * contains on every get (:224), one key at a time, on a filter sized from the write buffer
 * (mem.rs:188-191: 51 200 bytes / 100 = 512 entries at p = 1e-4 -> m = 9815, k = 19).  This
 * times those calls through the C ABI exactly as a Rust binding would make them (one key per
 * call, n = 1, len_prefix = 1), for the two residencies:
 *   host    : vbf_filter_new(..., VBF_DEVICE_HOST, ...) -- bits in host memory, CPU hashing
 *   device  : vbf_filter_new(..., 0, ...)               -- bits in HBM, one staged launch per call
 * and checks that both end with the same words (the CPU rounds against the kernels).
 *
 * Then the read path against a compaction-built filter (sized.rs:192-193: new(1e-4, n) + one
 * batch build of n keys, bits in HBM): every get probes each in-range SST's filter with one key
 * (key_range/range.rs:130,136,171).  Those single-key contains answer from the filter's host
 * mirror (VBF_MIRROR_LAZY, the default; the first get after the build pays one D2H), timed
 * against the same gets with the mirror off (one staged GPU round trip each).
 *
 * usage: memtable_latency [N_KEYS [DEVICE_KEYS [SST_KEYS]]]   (defaults 200000, 2000, 1000000)
 * prints one JSON line; exit 1 on any library failure or mismatch. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "vbf.h"

static void check(int rc, const char* what) {
    if (rc != VBF_OK) {
        fprintf(stderr, "%s failed (%d): %s\n", what, rc, vbf_last_error());
        exit(1);
    }
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int cmp_d(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

/* key j: "user:" + 11 decimal digits (16 bytes, like a short application key) */
static void make_key(uint64_t j, char out[17]) {
    snprintf(out, 17, "user:%011llu", (unsigned long long)(j % 100000000000ull));
}

struct lat {
    double put_mean_us, put_p50_us, put_p99_us, get_mean_us, get_p50_us, get_p99_us;
    uint32_t n_elements;
};

/* `n` puts (contains, then set when absent: mem.rs:209-211), then `n` gets of the same keys and
 * `n` gets of absent keys (mem.rs:224).  Per-call times in microseconds. */
static struct lat run(vbf_filter* f, uint64_t n) {
    double* t = malloc(sizeof(double) * 2 * n);
    double put_sum = 0, get_sum = 0;
    char key[17];
    for (uint64_t j = 0; j < n; ++j) {
        make_key(j, key);
        const uint64_t off[2] = {0, 16};
        uint8_t hit = 0;
        const double a = now_s();
        check(vbf_filter_contains_host(f, (const uint8_t*)key, off, 0, 1, 1, &hit), "contains");
        if (!hit) check(vbf_filter_set_host(f, (const uint8_t*)key, off, 0, 1, 1), "set");
        t[j] = (now_s() - a) * 1e6;
        put_sum += t[j];
    }
    struct lat r;
    qsort(t, n, sizeof(double), cmp_d);
    r.put_mean_us = put_sum / (double)n;
    r.put_p50_us = t[n / 2];
    r.put_p99_us = t[(n * 99) / 100];
    for (uint64_t j = 0; j < 2 * n; ++j) {
        make_key(j, key);  /* keys n..2n-1 were never put */
        const uint64_t off[2] = {0, 16};
        uint8_t hit = 0;
        const double a = now_s();
        check(vbf_filter_contains_host(f, (const uint8_t*)key, off, 0, 1, 1, &hit), "contains");
        t[j] = (now_s() - a) * 1e6;
        get_sum += t[j];
        if (j < n && !hit) {
            fprintf(stderr, "false negative for key %llu\n", (unsigned long long)j);
            exit(1);
        }
    }
    qsort(t, 2 * n, sizeof(double), cmp_d);
    r.get_mean_us = get_sum / (double)(2 * n);
    r.get_p50_us = t[n];
    r.get_p99_us = t[(2 * n * 99) / 100];
    r.n_elements = vbf_filter_num_elements(f);
    free(t);
    return r;
}

struct glat {
    uint64_t n, false_neg;
    double mean_us, p50_us, p99_us, first_us, fp_rate;
    uint8_t* hits;
};

/* `n` gets against a filter holding keys 0..n_set-1: even calls a present key (spread over the
 * set), odd calls an absent one.  The key sequence depends only on the call index. */
static struct glat gets(vbf_filter* f, uint64_t n_set, uint64_t n) {
    struct glat r = {n, 0, 0, 0, 0, 0, 0, malloc(n)};
    double* t = malloc(sizeof(double) * n);
    double sum = 0;
    uint64_t fp = 0, neg = 0;
    char key[17];
    for (uint64_t i = 0; i < n; ++i) {
        const int present = (i & 1) == 0;
        make_key(present ? (i * 7919u) % n_set : n_set + i, key);
        uint8_t hit = 0;
        const double a = now_s();
        check(vbf_filter_contains_host(f, (const uint8_t*)key, NULL, 16, 1, 1, &hit), "contains");
        t[i] = (now_s() - a) * 1e6;
        sum += t[i];
        r.hits[i] = hit;
        if (present && !hit) r.false_neg++;
        if (!present) {
            neg++;
            fp += hit;
        }
    }
    r.first_us = t[0];
    r.mean_us = sum / (double)n;
    qsort(t, n, sizeof(double), cmp_d);
    r.p50_us = t[n / 2];
    r.p99_us = t[(n * 99) / 100];
    r.fp_rate = neg ? (double)fp / (double)neg : 0.0;
    free(t);
    return r;
}

int main(int argc, char** argv) {
    const uint64_t n_host = argc > 1 ? strtoull(argv[1], NULL, 10) : 200000;
    const uint64_t n_dev = argc > 2 ? strtoull(argv[2], NULL, 10) : 2000;
    const double p = 1e-4;
    const uint64_t entries = 51200 / 100; /* mem.rs:188-191 with the default 50 KiB buffer */

    vbf_filter* hf = NULL;
    check(vbf_filter_new(p, entries, VBF_DEVICE_HOST, &hf), "vbf_filter_new(host)");
    const uint32_t m = vbf_filter_num_bits(hf), k = vbf_filter_num_hash_functions(hf);
    struct lat h = run(hf, n_host);

    int ndev = 0;
    if (vbf_device_count(&ndev) != VBF_OK || ndev < 1) { /* host residency needs no GPU */
        printf("{\"m\": %u, \"k\": %u, \"host\": {\"keys\": %llu, \"put_us\": {\"mean\": %.3f, \"p50\": %.3f, "
               "\"p99\": %.3f}, \"get_us\": {\"mean\": %.3f, \"p50\": %.3f, \"p99\": %.3f}, \"n_elements\": %u}, "
               "\"device\": null}\n",
               m, k, (unsigned long long)n_host, h.put_mean_us, h.put_p50_us, h.put_p99_us, h.get_mean_us,
               h.get_p50_us, h.get_p99_us, h.n_elements);
        vbf_filter_free(hf);
        return 0;
    }
    vbf_filter* df = NULL;
    check(vbf_filter_new(p, entries, 0, &df), "vbf_filter_new(device 0)");
    struct lat d = run(df, n_dev);

    /* the same first n_dev puts into a fresh host filter: words must equal the device's */
    vbf_filter* h2 = NULL;
    check(vbf_filter_new(p, entries, VBF_DEVICE_HOST, &h2), "vbf_filter_new(host)");
    (void)run(h2, n_dev);
    const uint64_t nw = (m + 31) / 32;
    uint32_t* wh = malloc(nw * 4);
    uint32_t* wd = malloc(nw * 4);
    check(vbf_filter_words_to_host(h2, wh, nw), "words(host)");
    check(vbf_filter_words_to_host(df, wd, nw), "words(device)");
    const int same = memcmp(wh, wd, nw * 4) == 0 && vbf_filter_num_elements(h2) == vbf_filter_num_elements(df);

    /* read path on a compaction-built, device-resident filter */
    const uint64_t n_sst = argc > 3 ? strtoull(argv[3], NULL, 10) : 1000000;
    char* packed = malloc(n_sst * 16);
    char key[17];
    for (uint64_t j = 0; j < n_sst; ++j) {
        make_key(j, key);
        memcpy(packed + j * 16, key, 16);
    }
    vbf_filter* cf = NULL;
    check(vbf_filter_new(p, n_sst, 0, &cf), "vbf_filter_new(compaction)");
    double a = now_s();
    check(vbf_filter_set_host(cf, (const uint8_t*)packed, NULL, 16, n_sst, 1), "build_filter_from_entries");
    const double build_ms = (now_s() - a) * 1e3;
    a = now_s();
    struct glat mir = gets(cf, n_sst, 200000);  /* first get fills the mirror */
    const double mir_total_s = now_s() - a;
    check(vbf_filter_set_mirror(cf, VBF_MIRROR_OFF), "set_mirror(off)");
    struct glat gpu = gets(cf, n_sst, 2000);
    check(vbf_filter_set_mirror(cf, VBF_MIRROR_LAZY), "set_mirror(lazy)");

    printf("{\"m\": %u, \"k\": %u, \"host\": {\"keys\": %llu, \"put_us\": {\"mean\": %.3f, \"p50\": %.3f, \"p99\": %.3f}, "
           "\"get_us\": {\"mean\": %.3f, \"p50\": %.3f, \"p99\": %.3f}, \"n_elements\": %u}, "
           "\"device\": {\"keys\": %llu, \"put_us\": {\"mean\": %.3f, \"p50\": %.3f, \"p99\": %.3f}, "
           "\"get_us\": {\"mean\": %.3f, \"p50\": %.3f, \"p99\": %.3f}, \"n_elements\": %u}, "
           "\"host_words_equal_device_words\": %s, "
           "\"compaction_filter\": {\"keys\": %llu, \"m\": %u, \"k\": %u, \"build_ms\": %.3f, "
           "\"get_us_mirror\": {\"gets\": %llu, \"mean\": %.3f, \"p50\": %.3f, \"p99\": %.3f, \"first\": %.1f, "
           "\"wall_s\": %.3f}, "
           "\"get_us_gpu\": {\"gets\": %llu, \"mean\": %.3f, \"p50\": %.3f, \"p99\": %.3f}, "
           "\"false_negatives\": %llu, \"fp_rate\": %.6f}}\n",
           m, k, (unsigned long long)n_host, h.put_mean_us, h.put_p50_us, h.put_p99_us, h.get_mean_us, h.get_p50_us,
           h.get_p99_us, h.n_elements, (unsigned long long)n_dev, d.put_mean_us, d.put_p50_us, d.put_p99_us,
           d.get_mean_us, d.get_p50_us, d.get_p99_us, d.n_elements, same ? "true" : "false",
           (unsigned long long)n_sst, vbf_filter_num_bits(cf), vbf_filter_num_hash_functions(cf), build_ms,
           (unsigned long long)mir.n, mir.mean_us, mir.p50_us, mir.p99_us, mir.first_us, mir_total_s,
           (unsigned long long)gpu.n, gpu.mean_us, gpu.p50_us, gpu.p99_us,
           (unsigned long long)(mir.false_neg + gpu.false_neg), mir.fp_rate);
    const int ok_all = same && mir.false_neg == 0 && gpu.false_neg == 0 && memcmp(mir.hits, gpu.hits, gpu.n) == 0;
    vbf_filter_free(hf);
    vbf_filter_free(df);
    vbf_filter_free(h2);
    vbf_filter_free(cf);
    free(wh);
    free(wd);
    free(packed);
    free(mir.hits);
    free(gpu.hits);
    return ok_all ? 0 : 1;
}
