/*
 * c4_call_c.c -- the synchronous C4 call timed from C (no Python, no
 * ctypes): 256 hipMalloc'ed iput-shaped segments (NC_SHORT from short,
 * NC_FLOAT from float, 2^20 elements each, BASELINE config 4), W untimed
 * calls, then K calls on the wall clock, then K more with the library's
 * kernel events (pncx_dev_batch_timing), and the same for a trivial batch
 * of one 1-element segment (the floor of a synchronous call).  Separates
 * the library's per-call overhead from bench.py's Python loop (DESIGN §0
 * item 4).  Not product code.
 *
 *   gcc -O2 -I include -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/c4_call_c.c -o tools/c4_call_c \
 *       -Lpnetcdf_amd/lib -lpncx -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN/../pnetcdf_amd/lib' \
 *       -Wl,-rpath,/opt/rocm/lib
 *   tools/c4_call_c [K] [W]
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pncx.h"

static double now_ms(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

static int run(const pncx_seg *segs, int nseg, int k, int w, double *call_ms, double *kern_ms)
{
    int *st = (int *)calloc((size_t)nseg, sizeof(int)), i, rc = 0;
    double t0, tot = 0;
    long long calls = 0;
    for (i = 0; i < w && !rc; i++) rc = pncx_dev_batch(segs, nseg, st, NULL);
    t0 = now_ms();
    for (i = 0; i < k && !rc; i++) rc = pncx_dev_batch(segs, nseg, st, NULL);
    *call_ms = (now_ms() - t0) / k;
    pncx_dev_batch_timing(1);
    for (i = 0; i < k && !rc; i++) rc = pncx_dev_batch(segs, nseg, st, NULL);
    if (!rc) rc = pncx_dev_batch_kernel_ms(&tot, &calls);
    pncx_dev_batch_timing(0);
    *kern_ms = calls ? tot / (double)calls : -1;
    free(st);
    return rc;
}

int main(int argc, char **argv)
{
    const int k = argc > 1 ? atoi(argv[1]) : 200, w = argc > 2 ? atoi(argv[2]) : 20;
    const long long nel = 1 << 20;
    const int nvar = 256;
    pncx_seg segs[256], one;
    static unsigned char fill_s[8] = {0x01, 0x80}, fill_f[8];
    double cm, km, cm1, km1;
    int v, rc;
    memset(fill_f, 0, sizeof fill_f);
    for (v = 0; v < nvar; v++) {
        const int esz = v % 2 == 0 ? 2 : 4;
        void *x = NULL, *ib = NULL;
        if (hipMalloc(&x, (size_t)nel * esz) != hipSuccess || hipMalloc(&ib, (size_t)nel * esz) != hipSuccess ||
            hipMemset(ib, v, (size_t)nel * esz) != hipSuccess) {
            fprintf(stderr, "hipMalloc failed\n");
            return 2;
        }
        segs[v].dir = PNCX_PUT;
        segs[v].cdf_ver = 5;
        segs[v].xtype = esz == 2 ? NC_SHORT : NC_FLOAT;
        segs[v].itype = esz == 2 ? PNCX_ITYPE_SHORT : PNCX_ITYPE_FLOAT;
        segs[v].nelems = nel;
        segs[v].xbuf = x;
        segs[v].ibuf = ib;
        segs[v].fillp = esz == 2 ? (const void *)fill_s : (const void *)fill_f;
    }
    one = segs[1];
    one.nelems = 1;
    if ((rc = run(segs, nvar, k, w, &cm, &km)) != 0 || (rc = run(&one, 1, k, w, &cm1, &km1)) != 0) {
        fprintf(stderr, "pncx_dev_batch -> %d\n", rc);
        return 1;
    }
    printf("{\"c4_call_ms\": %.4f, \"c4_kernel_ms\": %.4f, \"c4_call_over_kernel\": %.4f, "
           "\"trivial_call_ms\": %.4f, \"trivial_kernel_ms\": %.4f, \"calls\": %d}\n",
           cm, km, cm / km, cm1, km1, k);
    return 0;
}
