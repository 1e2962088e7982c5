// c1_first_probe.hip -- first-touch cost of C1 under the reference's own
// access pattern (benchmarks/C/pnetcdf_put_vara.c:193-209: each record of a
// record variable written exactly once, appended past the end of the file;
// then each record read once).  Not product code: it decides how the
// product's host-buffer record puts are built.
//
//   hipcc --offload-arch=gfx950 -O2 -fopenmp -o tools/c1_first_probe tools/c1_first_probe.hip \
//         -Lpnetcdf_amd/lib -lpncx -Wl,-rpath,'$ORIGIN/../pnetcdf_amd/lib' 
//   tools/c1_first_probe /dev/shm/c1first.nc [bytes] [nrec]
//
// Every line is "name median_us mean_us min_us" over the nrec records.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <pthread.h>
#include <omp.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include <algorithm>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); exit(2); } } while (0)

static double now_us() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void report(const char *name, std::vector<double> v) {
    double s = 0;
    for (double x : v) s += x;
    std::sort(v.begin(), v.end());
    printf("%-52s %9.1f %9.1f %9.1f\n", name, v[v.size() / 2], s / v.size(), v[0]);
    fflush(stdout);
}

__global__ void __launch_bounds__(256) k_swap4(const uint4 *__restrict__ s, uint4 *__restrict__ d, long long nv) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= nv) return;
    uint4 v = s[i];
    v.x = __builtin_bswap32(v.x);
    v.y = __builtin_bswap32(v.y);
    v.z = __builtin_bswap32(v.z);
    v.w = __builtin_bswap32(v.w);
    d[i] = v;
}

// the product's I/O pool (pnetcdf_amd/csrc/pncx_io.h), linked from libpncx.so
extern "C" {
typedef struct pio_batch { pthread_mutex_t m; pthread_cond_t c; int pending; int err; } pio_batch;
void pio_batch_init(pio_batch *b);
void pio_batch_destroy(pio_batch *b);
int pio_wait(pio_batch *b);
int pio_prefetch(pio_batch *b, const void *p, size_t n, int parts);
}

static void cpu_swap4(uint32_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) p[i] = __builtin_bswap32(p[i]);
}

static const long long BASE = 512;      // the record section begins after a small header
static int g_fd;
static size_t g_bytes;

static void fresh() {
    static unsigned char hdr[BASE];
    if (ftruncate(g_fd, 0) != 0 || pwrite(g_fd, hdr, BASE, 0) != BASE) { perror("fresh"); exit(2); }
}

static off_t rec_off(int r) { return (off_t)(BASE + (long long)r * (long long)g_bytes); }

static void verify(const uint32_t *user, int nrec, const char *what) {
    std::vector<uint32_t> chk(g_bytes / 4);
    for (int r = 0; r < nrec; r += (nrec > 3 ? nrec / 3 : 1)) {
        if (pread(g_fd, chk.data(), g_bytes, rec_off(r)) != (ssize_t)g_bytes) { fprintf(stderr, "%s: short read\n", what); exit(3); }
        for (size_t i = 0; i < g_bytes / 4; i++)
            if (chk[i] != __builtin_bswap32(user[i])) { fprintf(stderr, "%s: mismatch rec %d at %zu\n", what, r, i); exit(3); }
    }
    struct stat st;
    fstat(g_fd, &st);
    if (st.st_size != BASE + (long long)nrec * (long long)g_bytes) {
        fprintf(stderr, "%s: file size %lld, expected %lld\n", what, (long long)st.st_size, BASE + (long long)nrec * (long long)g_bytes);
        exit(3);
    }
}

static void par_copy(void *dst, const void *src, size_t n, int T) {
    if (T <= 1) { memcpy(dst, src, n); return; }
    const size_t piece = ((n + T - 1) / T + 4095) & ~(size_t)4095;
#pragma omp parallel for num_threads(T) schedule(static, 1)
    for (int t = 0; t < T; t++) {
        const size_t a = (size_t)t * piece;
        if (a < n) memcpy((char *)dst + a, (const char *)src + a, std::min(piece, n - a));
    }
}

int main(int argc, char **argv) {
    const char *path = argc > 1 ? argv[1] : "/dev/shm/c1first.nc";
    g_bytes = argc > 2 ? (size_t)atoll(argv[2]) : (4u << 20);
    const int nrec = argc > 3 ? atoi(argv[3]) : 24;
    const bool v2 = argc > 4 && strcmp(argv[4], "v2") == 0;
    const bool v3 = argc > 4 && strcmp(argv[4], "v3") == 0;
    const size_t bytes = g_bytes, nv = bytes / 16;
    std::vector<double> t(nrec);
    hipStream_t s;
    CK(hipSetDevice(0));
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    g_fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
    if (g_fd < 0) { perror("open"); return 2; }
    omp_set_dynamic(0);
#pragma omp parallel num_threads(8)
    { (void)omp_get_thread_num(); }

    void *slot_def, *slot_coh, *slot_nc, *slot_reg_host;
    CK(hipHostMalloc(&slot_def, bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&slot_coh, bytes, hipHostMallocCoherent));
    CK(hipHostMalloc(&slot_nc, bytes, hipHostMallocNonCoherent));
    slot_reg_host = aligned_alloc(4096, bytes);
    memset(slot_reg_host, 1, bytes);
    CK(hipHostRegister(slot_reg_host, bytes, hipHostRegisterDefault));
    memset(slot_def, 1, bytes); memset(slot_coh, 1, bytes); memset(slot_nc, 1, bytes);
    uint32_t *user = (uint32_t *)malloc(bytes), *user2 = (uint32_t *)malloc(bytes);
    for (size_t i = 0; i < bytes / 4; i++) user[i] = (uint32_t)i * 2654435761u;
    memset(user2, 0, bytes);
    const int NCH_MAX = 16;
    hipEvent_t ev[NCH_MAX];
    for (int i = 0; i < NCH_MAX; i++) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    hipLaunchKernelGGL(k_swap4, dim3(1), dim3(256), 0, s, (const uint4 *)slot_def, (uint4 *)slot_coh, 0LL);
    CK(hipStreamSynchronize(s));
    printf("# bytes %zu records %d (us per record: median mean min)\n", bytes, nrec);

    // ---- P0: the reference's put (ncmpio_getput.m4:186-214,269-270 + the
    // collective numrecs write, :272-311): swap in place, pwrite, swap back,
    // 8-byte numrecs at offset 4 (CDF-5)
    fresh();
    for (int r = 0; r < nrec; r++) {
        double a = now_us();
        cpu_swap4(user, bytes / 4);
        if (pwrite(g_fd, user, bytes, rec_off(r)) != (ssize_t)bytes) return 2;
        cpu_swap4(user, bytes / 4);
        uint64_t nr = __builtin_bswap64((uint64_t)(r + 1));
        if (pwrite(g_fd, &nr, 8, 4) != 8) return 2;
        t[r] = now_us() - a;
    }
    report("P0 ref put (swap,pwrite,swap,numrecs)", t);
    verify(user, nrec, "P0");
    // the same onto existing pages (rewrite), for contrast
    for (int r = 0; r < nrec; r++) {
        double a = now_us();
        cpu_swap4(user, bytes / 4);
        if (pwrite(g_fd, user, bytes, rec_off(r)) != (ssize_t)bytes) return 2;
        cpu_swap4(user, bytes / 4);
        t[r] = now_us() - a;
    }
    report("P0r ref put rewrite (existing pages)", t);

    // ---- Q: a persistent shared mapping of the file (no populate); per
    // record: the file is extended to the record's end by a 1-byte fallocate
    // at end-1 (never shrinks, allocates one page), the GPU converts 4 chunks
    // user -> pinned slot, T threads pre-fault their slices of the record's
    // pages while the GPU runs (optional), then copy each chunk as it lands
    if (v2) {
        const int nch = 4;
        const size_t cb = bytes / nch, cnv = cb / 16;
        for (int pop = 0; pop < 2; pop++)
            for (int T : {1, 4, 8, 16}) {
                fresh();
                const size_t mlen = (size_t)BASE + (size_t)nrec * bytes + 4096;
                unsigned char *m = (unsigned char *)mmap(NULL, mlen, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_NORESERVE, g_fd, 0);
                if (m == MAP_FAILED) { perror("mmap"); return 2; }
                std::vector<double> tf(nrec), tw(nrec);
                for (int r = 0; r < nrec; r++) {
                    double a = now_us();
                    CK(hipHostRegister(user, bytes, hipHostRegisterDefault));
                    void *du, *ds;
                    CK(hipHostGetDevicePointer(&du, user, 0));
                    CK(hipHostGetDevicePointer(&ds, slot_def, 0));
                    for (int k = 0; k < nch; k++) {
                        hipLaunchKernelGGL(k_swap4, dim3((unsigned)((cnv + 255) / 256)), dim3(256), 0, s,
                                           (const uint4 *)((char *)du + k * cb), (uint4 *)((char *)ds + k * cb), (long long)cnv);
                        CK(hipEventRecord(ev[k], s));
                    }
                    const off_t off = rec_off(r);
                    double f0 = now_us();
                    struct stat st;
                    fstat(g_fd, &st);
                    if (st.st_size < off + (off_t)bytes && fallocate(g_fd, 0, off + (off_t)bytes - 1, 1) != 0) { perror("fallocate"); return 2; }
                    if (pop) {
                        const uintptr_t lo = ((uintptr_t)(m + off)) & ~(uintptr_t)4095;
                        const uintptr_t hi = ((uintptr_t)(m + off + bytes) + 4095) & ~(uintptr_t)4095;
                        const size_t npg = (hi - lo) / 4096, per = (npg + T - 1) / T;
#pragma omp parallel for num_threads(T) schedule(static, 1)
                        for (int tt = 0; tt < T; tt++) {
                            const size_t p0 = (size_t)tt * per, p1 = std::min(npg, p0 + per);
                            if (p0 < p1) madvise((void *)(lo + p0 * 4096), (p1 - p0) * 4096, MADV_POPULATE_WRITE);
                        }
                    }
                    tf[r] = now_us() - f0;
                    double w0 = now_us();
                    for (int k = 0; k < nch; k++) {
                        CK(hipEventSynchronize(ev[k]));
                        if (k == 0) w0 = now_us();
                        par_copy(m + off + k * cb, (char *)slot_def + k * cb, cb, T);
                    }
                    tw[r] = now_us() - w0;
                    CK(hipHostUnregister(user));
                    t[r] = now_us() - a;
                }
                char nm[160];
                snprintf(nm, sizeof nm, "Q 4ch mapping, extend 1B, %s, memcpy T=%d", pop ? "T-thread populate" : "faults in memcpy", T);
                report(nm, t);
                report("   .extend(+populate)", tf);
                report("   .copy after the first chunk landed", tw);
                double a = now_us();
                munmap(m, mlen);
                printf("   .munmap of the whole mapping: %.1f us (%.1f per record)\n", now_us() - a, (now_us() - a) / nrec);
                verify(user, nrec, nm);
            }
    }

    // ---- R: fallocate the record while the GPU converts, then pwrite per
    // chunk (P4), with helper threads that read chunk k+1 of the GPU-written
    // slot (pulling it out of DRAM into their caches) while the caller
    // pwrites chunk k; helpers placed on the caller's L3 siblings, or anywhere
    if (v3) {
        const int me = sched_getcpu();
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(me, &one);
        sched_setaffinity(0, sizeof one, &one);
        std::vector<int> sib;
        {
            char pth[128], buf[512];
            snprintf(pth, sizeof pth, "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", me);
            FILE *fp = fopen(pth, "r");
            if (fp && fgets(buf, sizeof buf, fp)) {
                char *q = buf;
                while (*q) {
                    int a = (int)strtol(q, &q, 10), b = a;
                    if (*q == '-') b = (int)strtol(q + 1, &q, 10);
                    for (int c = a; c <= b; c++) if (c != me) sib.push_back(c);
                    if (*q == ',') q++; else break;
                }
            }
            if (fp) fclose(fp);
            printf("# caller cpu %d, L3 siblings:", me);
            for (int c : sib) printf(" %d", c);
            printf("\n");
        }
        for (int nch : {4, 8})
            for (int mode = 0; mode < 6; mode++) {
                // 0: no helpers; 1: 3 helpers on L3 siblings; 2: 7 helpers on L3 siblings; 3: 3 helpers unpinned
                // 4: the product's I/O pool pulls (pio_prefetch, 3 parts); 5: the same, 1 part
                const int H = mode == 0 ? 0 : (mode == 2 ? 7 : 3);
                const size_t cb = bytes / nch, cnv = cb / 16;
                fresh();
                std::vector<double> tw(nrec);
                volatile unsigned long long sink = 0;
                for (int r = 0; r < nrec; r++) {
                    double a = now_us();
                    CK(hipHostRegister(user, bytes, hipHostRegisterDefault));
                    void *du, *ds;
                    CK(hipHostGetDevicePointer(&du, user, 0));
                    CK(hipHostGetDevicePointer(&ds, slot_def, 0));
                    for (int k = 0; k < nch; k++) {
                        hipLaunchKernelGGL(k_swap4, dim3((unsigned)((cnv + 255) / 256)), dim3(256), 0, s,
                                           (const uint4 *)((char *)du + k * cb), (uint4 *)((char *)ds + k * cb), (long long)cnv);
                        CK(hipEventRecord(ev[k], s));
                    }
                    const off_t off = rec_off(r);
                    if (fallocate(g_fd, 0, off, (off_t)bytes) != 0) { perror("fallocate"); return 2; }
                    double w0 = now_us();
                    if (mode >= 4) {
                        pio_batch tb[2];
                        pio_batch_init(&tb[0]);
                        pio_batch_init(&tb[1]);
                        const int parts = mode == 4 ? 3 : 1;
                        CK(hipEventSynchronize(ev[0]));
                        pio_prefetch(&tb[0], slot_def, cb, parts);
                        for (int k = 0; k < nch; k++) {
                            if (k + 1 < nch) {
                                CK(hipEventSynchronize(ev[k + 1]));
                                pio_prefetch(&tb[(k + 1) & 1], (char *)slot_def + (k + 1) * cb, cb, parts);
                            }
                            pio_wait(&tb[k & 1]);
                            if (pwrite(g_fd, (char *)slot_def + k * cb, cb, off + (off_t)(k * cb)) != (ssize_t)cb) return 2;
                        }
                        pio_batch_destroy(&tb[0]);
                        pio_batch_destroy(&tb[1]);
                    } else if (H == 0) {
                        for (int k = 0; k < nch; k++) {
                            CK(hipEventSynchronize(ev[k]));
                            if (pwrite(g_fd, (char *)slot_def + k * cb, cb, off + (off_t)(k * cb)) != (ssize_t)cb) return 2;
                        }
                    } else {
                        // thread 0 = the caller (pwrite), threads 1..H = helpers
#pragma omp parallel num_threads(H + 1)
                        {
                            const int id = omp_get_thread_num();
                            if (id > 0) {
                                cpu_set_t cs;
                                CPU_ZERO(&cs);
                                if (mode != 3 && !sib.empty()) CPU_SET(sib[(id - 1) % sib.size()], &cs);
                                else for (int c = 0; c < CPU_SETSIZE; c++) if (c != me) CPU_SET(c, &cs);
                                sched_setaffinity(0, sizeof cs, &cs);
                            }
                            unsigned long long acc = 0;
                            for (int k = 0; k <= nch; k++) {
                                // step k: helpers pull chunk k while the caller writes chunk k-1
                                if (id == 0) {
                                    if (k < nch) CK(hipEventSynchronize(ev[k]));
                                } 
#pragma omp barrier
                                if (id == 0) {
                                    if (k > 0 && pwrite(g_fd, (char *)slot_def + (k - 1) * cb, cb, off + (off_t)((k - 1) * cb)) != (ssize_t)cb) exit(2);
                                } else if (k < nch) {
                                    const size_t per = (cb / H + 63) & ~(size_t)63, a0 = (size_t)(id - 1) * per;
                                    const unsigned char *p = (const unsigned char *)slot_def + k * cb;
                                    for (size_t o = a0; o < std::min(cb, a0 + per); o += 64) acc += p[o];
                                }
#pragma omp barrier
                            }
                            if (acc == 1) sink = acc;
                        }
                    }
                    tw[r] = now_us() - w0;
                    CK(hipHostUnregister(user));
                    t[r] = now_us() - a;
                }
                (void)sink;
                static const char *mn[] = {"no helpers", "3 helpers on L3 siblings", "7 helpers on L3 siblings", "3 helpers unpinned",
                                           "libpncx pool pulls, 3 parts", "libpncx pool pulls, 1 part"};
                char nm[160];
                snprintf(nm, sizeof nm, "R %dch fallocate + pwrite/chunk, %s", nch, mn[mode]);
                report(nm, t);
                report("   .after fallocate (wait + pwrite)", tw);
                verify(user, nrec, nm);
            }
        cpu_set_t all;
        CPU_ZERO(&all);
        for (int c = 0; c < CPU_SETSIZE; c++) CPU_SET(c, &all);
        sched_setaffinity(0, sizeof all, &all);
    }

    // ---- P1: pwrite alone of a hot buffer, appended
    if (!v2 && !v3) {
    fresh();
    for (int r = 0; r < nrec; r++) {
        double a = now_us();
        if (pwrite(g_fd, user2, bytes, rec_off(r)) != (ssize_t)bytes) return 2;
        t[r] = now_us() - a;
    }
    report("P1 pwrite hot buffer, appended", t);
    fresh();
    for (int r = 0; r < nrec; r++) {
        double a = now_us();
        if (fallocate(g_fd, 0, rec_off(r), (off_t)bytes) != 0) return 2;
        t[r] = now_us() - a;
    }
    report("P1f fallocate alone, appended", t);
    for (int r = 0; r < nrec; r++) {
        double a = now_us();
        if (pwrite(g_fd, user2, bytes, rec_off(r)) != (ssize_t)bytes) return 2;
        t[r] = now_us() - a;
    }
    report("P1g pwrite hot into fallocated pages", t);

    // ---- P2: the GPU converts the whole record user -> pinned slot (zero
    // copy), then pwrite from the slot (cold); slot allocation variants
    struct { const char *name; void *slot; } slots[] = {
        {"P2 zc whole + pwrite, hipHostMalloc default", slot_def},
        {"P2 zc whole + pwrite, hipHostMalloc coherent", slot_coh},
        {"P2 zc whole + pwrite, hipHostMalloc noncoherent", slot_nc},
        {"P2 zc whole + pwrite, aligned_alloc+register", slot_reg_host}};
    for (auto &sl : slots) {
        fresh();
        std::vector<double> tk(nrec), tw(nrec);
        for (int r = 0; r < nrec; r++) {
            double a = now_us();
            CK(hipHostRegister(user, bytes, hipHostRegisterDefault));
            void *du, *ds;
            CK(hipHostGetDevicePointer(&du, user, 0));
            CK(hipHostGetDevicePointer(&ds, sl.slot, 0));
            hipLaunchKernelGGL(k_swap4, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, (const uint4 *)du, (uint4 *)ds, (long long)nv);
            CK(hipStreamSynchronize(s));
            double b = now_us();
            if (pwrite(g_fd, sl.slot, bytes, rec_off(r)) != (ssize_t)bytes) return 2;
            double c = now_us();
            CK(hipHostUnregister(user));
            t[r] = now_us() - a; tk[r] = b - a; tw[r] = c - b;
        }
        report(sl.name, t);
        report("   .kernel (reg+launch+sync)", tk);
        report("   .pwrite from the GPU-written slot", tw);
        verify(user, nrec, sl.name);
    }

    // ---- P3/P4/P5: chunked pipelines
    for (int nch : {4, 8}) {
        const size_t cb = bytes / nch, cnv = cb / 16;
        for (int variant = 0; variant < 6; variant++) {
            // 0: pwrite per chunk
            // 1: fallocate the record while the GPU converts, then pwrite per chunk
            // 2: persistent mapping, fallocate + MADV_POPULATE_WRITE while the GPU converts, 1-thread memcpy per chunk
            // 3: the same, 4 threads per chunk
            // 4: the same, 8 threads per chunk
            // 5: persistent mapping, fallocate + populate overlapped, wait all, 8-thread memcpy of the record
            fresh();
            unsigned char *m = nullptr;
            const size_t mlen = (size_t)BASE + (size_t)nrec * bytes + 4096;
            if (variant >= 2) {
                m = (unsigned char *)mmap(NULL, mlen, PROT_READ | PROT_WRITE, MAP_SHARED, g_fd, 0);
                if (m == MAP_FAILED) { perror("mmap"); return 2; }
            }
            const int T = variant == 3 ? 4 : (variant >= 4 ? 8 : 1);
            std::vector<double> tf(nrec);
            for (int r = 0; r < nrec; r++) {
                double a = now_us();
                CK(hipHostRegister(user, bytes, hipHostRegisterDefault));
                void *du, *ds;
                CK(hipHostGetDevicePointer(&du, user, 0));
                CK(hipHostGetDevicePointer(&ds, slot_def, 0));
                for (int k = 0; k < nch; k++) {
                    hipLaunchKernelGGL(k_swap4, dim3((unsigned)((cnv + 255) / 256)), dim3(256), 0, s,
                                       (const uint4 *)((char *)du + k * cb), (uint4 *)((char *)ds + k * cb), (long long)cnv);
                    CK(hipEventRecord(ev[k], s));
                }
                const off_t off = rec_off(r);
                double f0 = now_us();
                if (variant >= 1) {
                    if (fallocate(g_fd, 0, off, (off_t)bytes) != 0) { perror("fallocate"); return 2; }
                    if (variant >= 2) {
                        const uintptr_t lo = ((uintptr_t)(m + off)) & ~(uintptr_t)4095;
                        const uintptr_t hi = ((uintptr_t)(m + off + bytes) + 4095) & ~(uintptr_t)4095;
                        static int warned = 0;
                        if (madvise((void *)lo, hi - lo, MADV_POPULATE_WRITE) != 0 && !warned++) perror("madvise(POPULATE_WRITE)");
                    }
                }
                tf[r] = now_us() - f0;
                if (variant == 5) {
                    CK(hipEventSynchronize(ev[nch - 1]));
                    par_copy(m + off, slot_def, bytes, 8);
                } else {
                    for (int k = 0; k < nch; k++) {
                        CK(hipEventSynchronize(ev[k]));
                        if (variant <= 1) {
                            if (pwrite(g_fd, (char *)slot_def + k * cb, cb, off + (off_t)(k * cb)) != (ssize_t)cb) return 2;
                        } else {
                            par_copy(m + off + k * cb, (char *)slot_def + k * cb, cb, T);
                        }
                    }
                }
                CK(hipHostUnregister(user));
                t[r] = now_us() - a;
            }
            static const char *vn[] = {"pwrite per chunk", "fallocate overlapped + pwrite per chunk",
                                        "map+fallocate+populate overlapped, memcpy/chunk T=1",
                                        "map+fallocate+populate overlapped, memcpy/chunk T=4",
                                        "map+fallocate+populate overlapped, memcpy/chunk T=8",
                                        "map+fallocate+populate overlapped, wait all, memcpy T=8"};
            char nm[160];
            snprintf(nm, sizeof nm, "P%d %dch %s", 3 + variant, nch, vn[variant]);
            report(nm, t);
            if (variant >= 1) report("   .fallocate(+populate) on the CPU", tf);
            if (m) {
                double a = now_us();
                munmap(m, mlen);
                printf("   .munmap of the whole mapping: %.1f us\n", now_us() - a);
            }
            verify(user, nrec, nm);
        }
    }

    } // !v2
    // ---- gets over the records of the last put (pages exist)
    // G0: the reference's get (ncmpio_getput.m4:415-427,468-470,
    // ncmpio_util.c:884-888,934-936): malloc xbuf, pread, swap, memcpy, free
    for (int r = 0; r < nrec; r++) {
        double a = now_us();
        uint32_t *x = (uint32_t *)malloc(bytes);
        if (pread(g_fd, x, bytes, rec_off(r)) != (ssize_t)bytes) return 2;
        cpu_swap4(x, bytes / 4);
        memcpy(user2, x, bytes);
        free(x);
        t[r] = now_us() - a;
    }
    report("G0 ref get (malloc,pread,swap,memcpy,free)", t);
    for (int r = 0; r < nrec; r++) {
        double a = now_us();
        if (pread(g_fd, user2, bytes, rec_off(r)) != (ssize_t)bytes) return 2;
        cpu_swap4(user2, bytes / 4);
        t[r] = now_us() - a;
    }
    report("G0b pread into user + swap", t);
    for (int nch : {1, 4, 8}) {
        const size_t cb = bytes / nch, cnv = cb / 16;
        for (int variant = 0; variant < 3; variant++) {
            // 0: pread chunk k into the slot, launch its kernel
            // 1: persistent mapping, 4-thread memcpy chunk k into the slot, launch
            // 2: the same, 8 threads
            if (nch == 1 && variant > 0) continue;
            unsigned char *m = nullptr;
            const size_t mlen = (size_t)BASE + (size_t)nrec * bytes;
            if (variant >= 1) {
                m = (unsigned char *)mmap(NULL, mlen, PROT_READ, MAP_SHARED | MAP_POPULATE, g_fd, 0);
                if (m == MAP_FAILED) { perror("mmap"); return 2; }
            }
            memset(user2, 0, bytes);
            for (int r = 0; r < nrec; r++) {
                double a = now_us();
                CK(hipHostRegister(user2, bytes, hipHostRegisterDefault));
                void *du, *ds;
                CK(hipHostGetDevicePointer(&du, user2, 0));
                CK(hipHostGetDevicePointer(&ds, slot_def, 0));
                const off_t off = rec_off(r);
                for (int k = 0; k < nch; k++) {
                    if (variant == 0) {
                        if (pread(g_fd, (char *)slot_def + k * cb, cb, off + (off_t)(k * cb)) != (ssize_t)cb) return 2;
                    } else {
                        par_copy((char *)slot_def + k * cb, m + off + k * cb, cb, variant == 1 ? 4 : 8);
                    }
                    hipLaunchKernelGGL(k_swap4, dim3((unsigned)((cnv + 255) / 256)), dim3(256), 0, s,
                                       (const uint4 *)((char *)ds + k * cb), (uint4 *)((char *)du + k * cb), (long long)cnv);
                }
                CK(hipStreamSynchronize(s));
                CK(hipHostUnregister(user2));
                t[r] = now_us() - a;
            }
            for (size_t i = 0; i < bytes / 4; i++)
                if (user2[i] != user[i]) { fprintf(stderr, "get mismatch at %zu\n", i); return 3; }
            static const char *vn[] = {"pread per chunk + zc kernel", "mapping, 4-thread memcpy + zc kernel",
                                        "mapping, 8-thread memcpy + zc kernel"};
            char nm[160];
            snprintf(nm, sizeof nm, "G%d %dch %s", 1 + variant, nch, vn[variant]);
            report(nm, t);
            if (m) munmap(m, mlen);
        }
    }
    close(g_fd);
    unlink(path);
    printf("# ok\n");
    return 0;
}
