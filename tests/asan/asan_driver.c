/* Host-side AddressSanitizer driver for the C-ABI ("ASan host build of the C-ABI").
 * Built by tests/asan/build.sh with capi.cpp and gen.cpp instrumented (-Xarch_host
 * -fsanitize=address,undefined; device code untouched) and linked with the regular
 * graph/consensus/cd objects.  Runs on a CPU-only host: every entry point's argument checks
 * and error paths, the native edge-list parser on the golden fixtures (and on malformed and
 * long-line inputs), and the LFR/SBM generators; fc_create's no-device path.  Exit 0 = clean. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/fastconsensus_amd.h"

static int fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) { fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); ++fails; } \
    } while (0)

static void parse(const char* path, int expect_ok) {
    int64_t n = -1, m = -1;
    int rc = fc_read_edgelist(path, &n, &m, NULL, NULL, NULL);
    if (!expect_ok) { CHECK(rc != FC_OK); CHECK(strlen(fc_last_error()) > 0); return; }
    CHECK(rc == FC_OK);
    if (rc != FC_OK) return;
    int64_t* labels = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n ? n : 1));
    int32_t* u = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m ? m : 1));
    int32_t* v = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m ? m : 1));
    int64_t n2 = 0, m2 = 0;
    CHECK(fc_read_edgelist(path, &n2, &m2, labels, u, v) == FC_OK);
    CHECK(n2 == n && m2 == m);
    for (int64_t i = 0; i < m; ++i) CHECK(u[i] >= 0 && u[i] < n && v[i] >= 0 && v[i] < n);
    printf("parsed %s: n=%lld m=%lld\n", path, (long long)n, (long long)m);
    free(labels); free(u); free(v);
}

static void write_file(const char* path, const char* text) {
    FILE* f = fopen(path, "w");
    fputs(text, f);
    fclose(f);
}

int main(int argc, char** argv) {
    const char* golden = argc > 1 ? argv[1] : "tests/golden";
    const char* tmp = argc > 2 ? argv[2] : "/tmp";
    printf("%s\n", fc_version());
    /* no device here: fc_create fails cleanly and leaves an error message */
    fc_ctx* ctx = NULL;
    const int crc = fc_create(0, 1, &ctx);
    if (crc != FC_OK) { CHECK(ctx == NULL && strlen(fc_last_error()) > 0); printf("fc_create: %d %s\n", crc, fc_last_error()); }
    else fc_destroy(ctx);
    CHECK(fc_create(0, 1, NULL) != FC_OK);
    /* null contexts are rejected by every stateful entry point */
    fc_destroy(NULL);
    CHECK(fc_load_graph(NULL, 2, 1, NULL, NULL) != FC_OK);
    CHECK(fc_run(NULL, 0, 4, 0.2, 0.02, NULL, NULL) != FC_OK);
    CHECK(fc_set_option(NULL, FC_OPT_SEED, 1) != FC_OK);
    CHECK(fc_set_params(NULL, 0, 0, 0) != FC_OK);
    /* parser: fixtures, comments, extra columns, malformed lines, a long line, missing file */
    char path[4096];
    snprintf(path, sizeof path, "%s/karate_club.txt", golden);
    parse(path, 1);
    snprintf(path, sizeof path, "%s/lfr1k_mu04.txt", golden);
    parse(path, 1);
    snprintf(path, sizeof path, "%s/fc_asan_ok.txt", tmp);
    write_file(path, "# header\n1 2\n2 3 0.5\n\n3\t4 {'weight': 1}\n4 1 # tail\n");
    parse(path, 1);
    snprintf(path, sizeof path, "%s/fc_asan_bad.txt", tmp);
    write_file(path, "1 2\nx y\n");
    parse(path, 0);
    snprintf(path, sizeof path, "%s/fc_asan_long.txt", tmp);
    {
        FILE* f = fopen(path, "w");
        fputs("1 2 ", f);
        for (int i = 0; i < 3000; ++i) fputs("7 ", f);   /* > 4 KiB line of extra columns */
        fputs("\n2 3\n", f);
        fclose(f);
    }
    {   /* parses or reports an error; either way no out-of-bounds access */
        int64_t n = 0, m = 0;
        (void)fc_read_edgelist(path, &n, &m, NULL, NULL, NULL);
    }
    parse("/nonexistent/fc_asan_missing.txt", 0);
    /* generators: bad arguments, then small graphs, then a capacity too small to hold them */
    int64_t m = 0;
    CHECK(fc_generate_lfr(1, 3, 1.5, 0.5, 20, 50, 20, 100, 1, 0, NULL, NULL, &m, NULL) != FC_OK);
    CHECK(fc_generate_sbm(10, 3, 5, 5, 1, 0, NULL, NULL, &m) != FC_OK);
    const int64_t n = 10000, cap = 400000;
    int32_t* u = (int32_t*)malloc(sizeof(int32_t) * cap);
    int32_t* v = (int32_t*)malloc(sizeof(int32_t) * cap);
    int32_t* planted = (int32_t*)malloc(sizeof(int32_t) * n);
    CHECK(fc_generate_lfr(n, 3, 1.5, 0.5, 20, 50, 20, 100, 42, cap, u, v, &m, planted) == FC_OK);
    printf("lfr n=%lld m=%lld\n", (long long)n, (long long)m);
    for (int64_t i = 0; i < m; ++i) CHECK(u[i] >= 0 && u[i] < n && v[i] >= 0 && v[i] < n && u[i] != v[i]);
    CHECK(fc_generate_sbm(n, 100, 10, 10, 42, cap, u, v, &m) == FC_OK);
    printf("sbm n=%lld m=%lld\n", (long long)n, (long long)m);
    int rc = fc_generate_lfr(n, 3, 1.5, 0.5, 20, 50, 20, 100, 42, 1000, u, v, &m, planted);
    printf("lfr with cap 1000: rc=%d m=%lld\n", rc, (long long)m);
    free(u); free(v); free(planted);
    printf(fails ? "ASAN DRIVER: %d checks failed\n" : "ASAN DRIVER: clean\n", fails);
    return fails ? 1 : 0;
}
