// c1_probe.hip -- cost of every piece the C1 host-boundary call could be
// built from (BASELINE configs[0]: 2^20 NC_INT put_vara + get_vara, 4 MiB,
// one rank, tmpfs).  Not product code: it decides how the product's
// host-buffer path is built (DESIGN.md §6 "C1 phases").
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/c1_probe tools/c1_probe.hip
//   tools/c1_probe /dev/shm/c1probe.nc [bytes] [reps]
//
// Every line is "name median_us min_us" over reps repetitions.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); exit(2); } } while (0)

static double now_us() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void report(const char *name, std::vector<double> &v) {
    std::sort(v.begin(), v.end());
    printf("%-44s %9.1f %9.1f\n", name, v[v.size() / 2], v[0]);
    fflush(stdout);
}

// 4-byte swap, one 16-byte vector per lane, plain global accesses: src and
// dst may be device memory or host memory mapped into the GPU (zero copy)
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

// four 16-byte vectors per lane, all loads issued before the stores
__global__ void __launch_bounds__(256) k_swap4_x4(const uint4 *__restrict__ s, uint4 *__restrict__ d, long long nv) {
    const long long i0 = ((long long)blockIdx.x * 256) * 4 + threadIdx.x;
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const long long i = i0 + u * 256;
        if (i < nv) v[u] = s[i];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const long long i = i0 + u * 256;
        if (i < nv) {
            uint4 w = v[u];
            w.x = __builtin_bswap32(w.x); w.y = __builtin_bswap32(w.y);
            w.z = __builtin_bswap32(w.z); w.w = __builtin_bswap32(w.w);
            d[i] = w;
        }
    }
}

__global__ void k_empty() {}

static void cpu_swap4(uint32_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) p[i] = __builtin_bswap32(p[i]);
}

int main(int argc, char **argv) {
    const char *path = argc > 1 ? argv[1] : "/dev/shm/c1probe.nc";
    const size_t bytes = argc > 2 ? (size_t)atoll(argv[2]) : (4u << 20);
    const int reps = argc > 3 ? atoi(argv[3]) : 41;
    const size_t nv = bytes / 16;
    const unsigned grid = (unsigned)((nv + 255) / 256);
    std::vector<double> t(reps);
    hipStream_t s;
    CK(hipSetDevice(0));
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
    CK(hipStreamSynchronize(s));

    void *dbuf, *dbuf2, *pin, *pin2;
    CK(hipMalloc(&dbuf, bytes));
    CK(hipMalloc(&dbuf2, bytes));
    CK(hipHostMalloc(&pin, bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&pin2, bytes, hipHostMallocDefault));
    uint32_t *user = (uint32_t *)malloc(bytes), *user2 = (uint32_t *)malloc(bytes);
    for (size_t i = 0; i < bytes / 4; i++) user[i] = (uint32_t)i * 2654435761u;
    memset(user2, 0, bytes);
    memset(pin, 1, bytes);
    memset(pin2, 1, bytes);
    printf("# bytes %zu reps %d (us: median min)\n", bytes, reps);

    // ---- launch / sync floors
    for (int r = 0; r < reps; r++) { double a = now_us(); CK(hipStreamSynchronize(s)); t[r] = now_us() - a; }
    report("sync_idle_stream", t);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        CK(hipStreamSynchronize(s));
        t[r] = now_us() - a;
    }
    report("empty_kernel_launch_sync", t);
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        CK(hipEventRecord(ev, s));
        while (hipEventQuery(ev) == hipErrorNotReady) {}
        t[r] = now_us() - a;
    }
    report("empty_kernel_event_spin", t);

    // ---- device-resident kernel
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)dbuf, (uint4 *)dbuf2, (long long)nv);
        CK(hipStreamSynchronize(s));
        t[r] = now_us() - a;
    }
    report("swap4_device_launch_sync", t);

    // ---- registration
    std::vector<double> t2(reps);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        CK(hipHostRegister(user, bytes, hipHostRegisterDefault));
        double b = now_us();
        CK(hipHostUnregister(user));
        t[r] = b - a;
        t2[r] = now_us() - b;
    }
    report("host_register", t);
    report("host_unregister", t2);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        CK(hipHostRegister(user, bytes, hipHostRegisterMapped));
        double b = now_us();
        CK(hipHostUnregister(user));
        t[r] = b - a;
        t2[r] = now_us() - b;
    }
    report("host_register_mapped", t);
    report("host_unregister_mapped", t2);
    hipPointerAttribute_t at;
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        (void)hipPointerGetAttributes(&at, user);
        (void)hipGetLastError();
        t[r] = now_us() - a;
    }
    report("pointer_get_attributes_pageable", t);

    // ---- copies (each with its stream sync)
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        CK(hipMemcpyAsync(dbuf, user, bytes, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        t[r] = now_us() - a;
    }
    report("h2d_pageable", t);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        CK(hipMemcpyAsync(user2, dbuf, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        t[r] = now_us() - a;
    }
    report("d2h_pageable", t);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        CK(hipMemcpyAsync(dbuf, pin, bytes, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        t[r] = now_us() - a;
    }
    report("h2d_pinned", t);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        CK(hipMemcpyAsync(pin, dbuf, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        t[r] = now_us() - a;
    }
    report("d2h_pinned", t);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        CK(hipMemcpyAsync(dbuf, pin, bytes, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)dbuf, (uint4 *)dbuf2, (long long)nv);
        CK(hipMemcpyAsync(pin2, dbuf2, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        t[r] = now_us() - a;
    }
    report("staged_pinned_h2d_kernel_d2h", t);

    // ---- zero copy: the kernel reads and writes host memory over PCIe
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)pin, (uint4 *)pin2, (long long)nv);
        CK(hipStreamSynchronize(s));
        t[r] = now_us() - a;
    }
    report("zerocopy_pinned_to_pinned", t);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)pin, (uint4 *)dbuf, (long long)nv);
        CK(hipStreamSynchronize(s));
        t[r] = now_us() - a;
    }
    report("zerocopy_pinned_to_device", t);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)dbuf, (uint4 *)pin, (long long)nv);
        CK(hipStreamSynchronize(s));
        t[r] = now_us() - a;
    }
    report("zerocopy_device_to_pinned", t);
    {
        std::vector<double> t3(reps), t4(reps);
        for (int r = 0; r < reps; r++) {
            double a = now_us();
            CK(hipHostRegister(user, bytes, hipHostRegisterMapped));
            void *du = nullptr;
            CK(hipHostGetDevicePointer(&du, user, 0));
            double b = now_us();
            hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)du, (uint4 *)pin, (long long)nv);
            CK(hipStreamSynchronize(s));
            double c = now_us();
            CK(hipHostUnregister(user));
            double d = now_us();
            t[r] = d - a; t2[r] = b - a; t3[r] = c - b; t4[r] = d - c;
        }
        report("zc_put_total(reg+kernel+unreg)", t);
        report("zc_put.register", t2);
        report("zc_put.kernel_user_to_pinned", t3);
        report("zc_put.unregister", t4);
        uint32_t *chk = (uint32_t *)pin;
        for (size_t i = 0; i < bytes / 4; i++)
            if (chk[i] != __builtin_bswap32(user[i])) { fprintf(stderr, "zc put mismatch at %zu\n", i); return 3; }
        for (int r = 0; r < reps; r++) {
            double a = now_us();
            CK(hipHostRegister(user2, bytes, hipHostRegisterMapped));
            void *du = nullptr;
            CK(hipHostGetDevicePointer(&du, user2, 0));
            double b = now_us();
            hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)pin, (uint4 *)du, (long long)nv);
            CK(hipStreamSynchronize(s));
            double c = now_us();
            CK(hipHostUnregister(user2));
            double d = now_us();
            t[r] = d - a; t2[r] = b - a; t3[r] = c - b; t4[r] = d - c;
        }
        report("zc_get_total(reg+kernel+unreg)", t);
        report("zc_get.register", t2);
        report("zc_get.kernel_pinned_to_user", t3);
        report("zc_get.unregister", t4);
        for (size_t i = 0; i < bytes / 4; i++)
            if (user2[i] != user[i]) { fprintf(stderr, "zc get mismatch at %zu\n", i); return 3; }
        // chunked zero-copy put: k kernels with an event each (the write of
        // chunk j would start at event j)
        for (int nch : {2, 4, 8}) {
            std::vector<hipEvent_t> evs(nch);
            for (auto &e : evs) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            std::vector<double> first(reps);
            for (int r = 0; r < reps; r++) {
                CK(hipHostRegister(user, bytes, hipHostRegisterMapped));
                void *du = nullptr;
                CK(hipHostGetDevicePointer(&du, user, 0));
                double a = now_us();
                const size_t cv = nv / nch;
                for (int j = 0; j < nch; j++) {
                    hipLaunchKernelGGL(k_swap4, dim3((unsigned)((cv + 255) / 256)), dim3(256), 0, s,
                                       (const uint4 *)du + j * cv, (uint4 *)pin + j * cv, (long long)cv);
                    CK(hipEventRecord(evs[j], s));
                }
                CK(hipEventSynchronize(evs[0]));
                first[r] = now_us() - a;
                CK(hipEventSynchronize(evs[nch - 1]));
                t[r] = now_us() - a;
                CK(hipHostUnregister(user));
            }
            char nm[64];
            snprintf(nm, sizeof nm, "zc_put_%d_chunks.first_ready", nch);
            report(nm, first);
            snprintf(nm, sizeof nm, "zc_put_%d_chunks.all_ready", nch);
            report(nm, t);
            for (auto &e : evs) CK(hipEventDestroy(e));
        }
    }

    // ---- chunked staging patterns (what pncx_stage can be built from):
    // nch chunks of H2D -> kernel -> D2H between pinned buffers
    {
        hipStream_t s2, s3;
        CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
        std::vector<hipEvent_t> ek(16), eo(16);
        for (int j = 0; j < 16; j++) {
            CK(hipEventCreateWithFlags(&ek[j], hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&eo[j], hipEventDisableTiming));
        }
        std::vector<double> tenq(reps), tfirst(reps);
        for (int nch : {1, 2, 4, 8}) {
            const size_t cb = bytes / nch, cv = cb / 16;
            const unsigned g = (unsigned)((cv + 255) / 256);
            char *din = (char *)dbuf, *dout = (char *)dbuf2;
            // (a) one stream, chunks in sequence
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                for (int j = 0; j < nch; j++) {
                    CK(hipMemcpyAsync(din + j * cb, (char *)pin + j * cb, cb, hipMemcpyHostToDevice, s));
                    hipLaunchKernelGGL(k_swap4, dim3(g), dim3(256), 0, s, (const uint4 *)(din + j * cb),
                                       (uint4 *)(dout + j * cb), (long long)cv);
                    CK(hipMemcpyAsync((char *)pin2 + j * cb, dout + j * cb, cb, hipMemcpyDeviceToHost, s));
                    CK(hipEventRecord(eo[j], s));
                }
                tenq[r] = now_us() - a;
                CK(hipEventSynchronize(eo[0]));
                tfirst[r] = now_us() - a;
                CK(hipStreamSynchronize(s));
                t[r] = now_us() - a;
            }
            char nm[96];
            snprintf(nm, sizeof nm, "stage_1stream_%dch.total", nch); report(nm, t);
            snprintf(nm, sizeof nm, "stage_1stream_%dch.enqueue", nch); report(nm, tenq);
            snprintf(nm, sizeof nm, "stage_1stream_%dch.first", nch); report(nm, tfirst);
            // (b) two streams, chunks alternate
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                for (int j = 0; j < nch; j++) {
                    hipStream_t q = (j & 1) ? s2 : s;
                    CK(hipMemcpyAsync(din + j * cb, (char *)pin + j * cb, cb, hipMemcpyHostToDevice, q));
                    hipLaunchKernelGGL(k_swap4, dim3(g), dim3(256), 0, q, (const uint4 *)(din + j * cb),
                                       (uint4 *)(dout + j * cb), (long long)cv);
                    CK(hipMemcpyAsync((char *)pin2 + j * cb, dout + j * cb, cb, hipMemcpyDeviceToHost, q));
                    CK(hipEventRecord(eo[j], q));
                }
                tenq[r] = now_us() - a;
                CK(hipEventSynchronize(eo[0]));
                tfirst[r] = now_us() - a;
                CK(hipStreamSynchronize(s));
                CK(hipStreamSynchronize(s2));
                t[r] = now_us() - a;
            }
            snprintf(nm, sizeof nm, "stage_2alt_%dch.total", nch); report(nm, t);
            snprintf(nm, sizeof nm, "stage_2alt_%dch.enqueue", nch); report(nm, tenq);
            snprintf(nm, sizeof nm, "stage_2alt_%dch.first", nch); report(nm, tfirst);
            // (c) in stream (H2D + kernel), out stream (D2H) joined by events
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                for (int j = 0; j < nch; j++) {
                    CK(hipMemcpyAsync(din + j * cb, (char *)pin + j * cb, cb, hipMemcpyHostToDevice, s));
                    hipLaunchKernelGGL(k_swap4, dim3(g), dim3(256), 0, s, (const uint4 *)(din + j * cb),
                                       (uint4 *)(dout + j * cb), (long long)cv);
                    CK(hipEventRecord(ek[j], s));
                    CK(hipStreamWaitEvent(s2, ek[j], 0));
                    CK(hipMemcpyAsync((char *)pin2 + j * cb, dout + j * cb, cb, hipMemcpyDeviceToHost, s2));
                    CK(hipEventRecord(eo[j], s2));
                }
                tenq[r] = now_us() - a;
                CK(hipEventSynchronize(eo[0]));
                tfirst[r] = now_us() - a;
                CK(hipStreamSynchronize(s2));
                t[r] = now_us() - a;
            }
            snprintf(nm, sizeof nm, "stage_inout_%dch.total", nch); report(nm, t);
            snprintf(nm, sizeof nm, "stage_inout_%dch.enqueue", nch); report(nm, tenq);
            snprintf(nm, sizeof nm, "stage_inout_%dch.first", nch); report(nm, tfirst);
            // (d) all H2D first on the in stream, kernels + D2H on the out stream
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                for (int j = 0; j < nch; j++) {
                    CK(hipMemcpyAsync(din + j * cb, (char *)pin + j * cb, cb, hipMemcpyHostToDevice, s));
                    CK(hipEventRecord(ek[j], s));
                }
                for (int j = 0; j < nch; j++) {
                    CK(hipStreamWaitEvent(s2, ek[j], 0));
                    hipLaunchKernelGGL(k_swap4, dim3(g), dim3(256), 0, s2, (const uint4 *)(din + j * cb),
                                       (uint4 *)(dout + j * cb), (long long)cv);
                    CK(hipMemcpyAsync((char *)pin2 + j * cb, dout + j * cb, cb, hipMemcpyDeviceToHost, s2));
                    CK(hipEventRecord(eo[j], s2));
                }
                tenq[r] = now_us() - a;
                CK(hipEventSynchronize(eo[0]));
                tfirst[r] = now_us() - a;
                CK(hipStreamSynchronize(s2));
                t[r] = now_us() - a;
            }
            snprintf(nm, sizeof nm, "stage_h2dfirst_%dch.total", nch); report(nm, t);
            snprintf(nm, sizeof nm, "stage_h2dfirst_%dch.enqueue", nch); report(nm, tenq);
            snprintf(nm, sizeof nm, "stage_h2dfirst_%dch.first", nch); report(nm, tfirst);
        }
        // (e) SDMA H2D on stream s, kernel writing the host result directly
        // (zero-copy store) on stream s2 after the chunk's H2D event
        for (int nch : {1, 2, 4, 8}) {
            const size_t cb = bytes / nch, cv = cb / 16;
            const unsigned g = (unsigned)((cv + 255) / 256);
            char *din = (char *)dbuf;
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                for (int j = 0; j < nch; j++) {
                    CK(hipMemcpyAsync(din + j * cb, (char *)pin + j * cb, cb, hipMemcpyHostToDevice, s));
                    CK(hipEventRecord(ek[j], s));
                    CK(hipStreamWaitEvent(s2, ek[j], 0));
                    hipLaunchKernelGGL(k_swap4, dim3(g), dim3(256), 0, s2, (const uint4 *)(din + j * cb),
                                       (uint4 *)((char *)pin2 + j * cb), (long long)cv);
                    CK(hipEventRecord(eo[j], s2));
                }
                tenq[r] = now_us() - a;
                CK(hipEventSynchronize(eo[0]));
                tfirst[r] = now_us() - a;
                CK(hipStreamSynchronize(s2));
                t[r] = now_us() - a;
            }
            char nm[96];
            snprintf(nm, sizeof nm, "stage_sdmain_zcout_%dch.total", nch); report(nm, t);
            snprintf(nm, sizeof nm, "stage_sdmain_zcout_%dch.first", nch); report(nm, tfirst);
            // (f) zero-copy in (kernel reads host into HBM... no: reads host,
            // writes HBM), SDMA D2H out after the chunk's kernel event
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                for (int j = 0; j < nch; j++) {
                    hipLaunchKernelGGL(k_swap4, dim3(g), dim3(256), 0, s, (const uint4 *)((char *)pin + j * cb),
                                       (uint4 *)(din + j * cb), (long long)cv);
                    CK(hipEventRecord(ek[j], s));
                    CK(hipStreamWaitEvent(s2, ek[j], 0));
                    CK(hipMemcpyAsync((char *)pin2 + j * cb, din + j * cb, cb, hipMemcpyDeviceToHost, s2));
                    CK(hipEventRecord(eo[j], s2));
                }
                tenq[r] = now_us() - a;
                CK(hipEventSynchronize(eo[0]));
                tfirst[r] = now_us() - a;
                CK(hipStreamSynchronize(s2));
                t[r] = now_us() - a;
            }
            snprintf(nm, sizeof nm, "stage_zcin_sdmaout_%dch.total", nch); report(nm, t);
            snprintf(nm, sizeof nm, "stage_zcin_sdmaout_%dch.first", nch); report(nm, tfirst);
            // (g) zero copy both ways, chunks on alternating streams
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                for (int j = 0; j < nch; j++) {
                    hipStream_t q = (j & 1) ? s2 : s;
                    hipLaunchKernelGGL(k_swap4, dim3(g), dim3(256), 0, q, (const uint4 *)((char *)pin + j * cb),
                                       (uint4 *)((char *)pin2 + j * cb), (long long)cv);
                    CK(hipEventRecord(eo[j], q));
                }
                tenq[r] = now_us() - a;
                CK(hipEventSynchronize(eo[0]));
                tfirst[r] = now_us() - a;
                CK(hipStreamSynchronize(s));
                CK(hipStreamSynchronize(s2));
                t[r] = now_us() - a;
            }
            snprintf(nm, sizeof nm, "stage_zc2alt_%dch.total", nch); report(nm, t);
            snprintf(nm, sizeof nm, "stage_zc2alt_%dch.first", nch); report(nm, tfirst);
        }
        // (h) zero-copy kernels with 4 vectors per lane
        {
            const unsigned g4 = (unsigned)((nv + 1023) / 1024);
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                hipLaunchKernelGGL(k_swap4_x4, dim3(g4), dim3(256), 0, s, (const uint4 *)pin, (uint4 *)pin2, (long long)nv);
                CK(hipStreamSynchronize(s));
                t[r] = now_us() - a;
            }
            report("zc_x4_pinned_to_pinned", t);
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                hipLaunchKernelGGL(k_swap4_x4, dim3(g4), dim3(256), 0, s, (const uint4 *)pin, (uint4 *)dbuf, (long long)nv);
                CK(hipStreamSynchronize(s));
                t[r] = now_us() - a;
            }
            report("zc_x4_pinned_to_device", t);
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                hipLaunchKernelGGL(k_swap4_x4, dim3(g4), dim3(256), 0, s, (const uint4 *)dbuf, (uint4 *)pin2, (long long)nv);
                CK(hipStreamSynchronize(s));
                t[r] = now_us() - a;
            }
            report("zc_x4_device_to_pinned", t);
        }
        // (i) H2D and D2H at the same time on two streams (full duplex?)
        for (int r = 0; r < reps; r++) {
            double a = now_us();
            CK(hipMemcpyAsync(dbuf, pin, bytes, hipMemcpyHostToDevice, s));
            CK(hipMemcpyAsync(pin2, dbuf2, bytes, hipMemcpyDeviceToHost, s2));
            CK(hipStreamSynchronize(s));
            CK(hipStreamSynchronize(s2));
            t[r] = now_us() - a;
        }
        report("h2d_and_d2h_concurrent", t);
        for (int r = 0; r < reps; r++) {
            double a = now_us();
            CK(hipMemcpyAsync(dbuf, pin, bytes, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s2, (const uint4 *)dbuf2, (uint4 *)pin2, (long long)nv);
            CK(hipStreamSynchronize(s));
            CK(hipStreamSynchronize(s2));
            t[r] = now_us() - a;
        }
        report("h2d_and_zcstore_concurrent", t);
        // enqueue costs alone (device-to-device, no wait)
        for (int r = 0; r < reps; r++) {
            double a = now_us();
            CK(hipMemcpyAsync(dbuf, pin, 4096, hipMemcpyHostToDevice, s));
            t[r] = now_us() - a;
            CK(hipStreamSynchronize(s));
        }
        report("enqueue.h2d_4k", t);
        for (int r = 0; r < reps; r++) {
            double a = now_us();
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
            t[r] = now_us() - a;
            CK(hipStreamSynchronize(s));
        }
        report("enqueue.kernel", t);
        for (int r = 0; r < reps; r++) {
            double a = now_us();
            CK(hipEventRecord(ek[0], s));
            t[r] = now_us() - a;
            CK(hipStreamSynchronize(s));
        }
        report("enqueue.event_record", t);
        for (int r = 0; r < reps; r++) {
            CK(hipEventRecord(ek[0], s));
            double a = now_us();
            CK(hipStreamWaitEvent(s2, ek[0], 0));
            t[r] = now_us() - a;
            CK(hipStreamSynchronize(s2));
        }
        report("enqueue.stream_wait_event", t);
    }

    // ---- CPU side
    for (int r = 0; r < reps; r++) { double a = now_us(); cpu_swap4(user, bytes / 4); t[r] = now_us() - a; }
    report("cpu_swap4_inplace", t);
    for (int r = 0; r < reps; r++) { double a = now_us(); memcpy(pin, user, bytes); t[r] = now_us() - a; }
    report("cpu_memcpy_user_to_pinned", t);

    // ---- file
    int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) { perror(path); return 2; }
    const off_t off = 512;
    if (ftruncate(fd, off + (off_t)bytes) != 0) { perror("ftruncate"); return 2; }
    if (pwrite(fd, user, bytes, off) != (ssize_t)bytes) { perror("pwrite"); return 2; }
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        if (pwrite(fd, pin, bytes, off) != (ssize_t)bytes) return 2;
        t[r] = now_us() - a;
    }
    report("pwrite_rewrite_from_pinned", t);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        if (pwrite(fd, user, bytes, off) != (ssize_t)bytes) return 2;
        t[r] = now_us() - a;
    }
    report("pwrite_rewrite_from_pageable", t);
    const long pg = sysconf(_SC_PAGESIZE);
    for (int flags : {MAP_SHARED, MAP_SHARED | MAP_POPULATE}) {
        for (int r = 0; r < reps; r++) {
            double a = now_us();
            unsigned char *m = (unsigned char *)mmap(NULL, bytes + off, PROT_WRITE, flags, fd, 0);
            if (m == MAP_FAILED) { perror("mmap"); return 2; }
            memcpy(m + off, pin, bytes);
            munmap(m, bytes + off);
            t[r] = now_us() - a;
        }
        report(flags & MAP_POPULATE ? "mmap_populate_memcpy_munmap" : "mmap_memcpy_munmap", t);
    }
    (void)pg;
    for (int nch : {4, 8}) {
        const size_t cb = bytes / nch;
        for (int r = 0; r < reps; r++) {
            double a = now_us();
            for (int j = 0; j < nch; j++)
                if (pwrite(fd, (char *)pin + j * cb, cb, off + (off_t)(j * cb)) != (ssize_t)cb) return 2;
            t[r] = now_us() - a;
        }
        char nm[64];
        snprintf(nm, sizeof nm, "pwrite_in_%d_pieces", nch);
        report(nm, t);
    }
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        if (pread(fd, pin, bytes, off) != (ssize_t)bytes) return 2;
        t[r] = now_us() - a;
    }
    report("pread_into_pinned", t);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        if (pread(fd, user2, bytes, off) != (ssize_t)bytes) return 2;
        t[r] = now_us() - a;
    }
    report("pread_into_pageable", t);
    // ---- the GPU writing/reading the file's page cache directly: a shared
    // mapping of the tmpfs file registered with HIP (zero-copy stores into
    // the file pages; no CPU copy of the converted bytes)
    {
        const off_t base = 0;                       /* the variable begins at off = 512 */
        const size_t span = (size_t)off + bytes;
        bool ok = true;
        std::vector<double> tm(reps), tr(reps), tk(reps), tu(reps);
        CK(hipHostRegister(user, bytes, hipHostRegisterMapped));
        void *duser = nullptr;
        CK(hipHostGetDevicePointer(&duser, user, 0));
        for (int r = 0; r < reps && ok; r++) {
            double a = now_us();
            unsigned char *m = (unsigned char *)mmap(NULL, span, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, base);
            if (m == MAP_FAILED) { perror("mmap"); ok = false; break; }
            double b = now_us();
            hipError_t e = hipHostRegister(m, span, hipHostRegisterMapped);
            if (e != hipSuccess) { printf("# file mapping register failed: %s\n", hipGetErrorString(e)); (void)hipGetLastError(); munmap(m, span); ok = false; break; }
            void *dm = nullptr;
            CK(hipHostGetDevicePointer(&dm, m, 0));
            double c = now_us();
            hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)duser, (uint4 *)((char *)dm + off), (long long)nv);
            CK(hipStreamSynchronize(s));
            double d = now_us();
            CK(hipHostUnregister(m));
            munmap(m, span);
            double e2 = now_us();
            t[r] = e2 - a; tm[r] = b - a; tr[r] = c - b; tk[r] = d - c; tu[r] = e2 - d;
        }
        if (ok) {
            report("fileput_zc.total(map+reg+kernel+unreg+unmap)", t);
            report("fileput_zc.mmap_populate", tm);
            report("fileput_zc.register", tr);
            report("fileput_zc.kernel_user_to_filepages", tk);
            report("fileput_zc.unregister_unmap", tu);
            std::vector<uint32_t> chk(bytes / 4);
            if (pread(fd, chk.data(), bytes, off) != (ssize_t)bytes) return 2;
            for (size_t i = 0; i < bytes / 4; i++)
                if (chk[i] != __builtin_bswap32(user[i])) { fprintf(stderr, "fileput mismatch at %zu\n", i); return 3; }
            printf("# fileput_zc verified\n");
            // persistent mapping: map + register once, the kernel per call
            unsigned char *m = (unsigned char *)mmap(NULL, span, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, base);
            CK(hipHostRegister(m, span, hipHostRegisterMapped));
            void *dm = nullptr;
            CK(hipHostGetDevicePointer(&dm, m, 0));
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)duser, (uint4 *)((char *)dm + off), (long long)nv);
                CK(hipStreamSynchronize(s));
                t[r] = now_us() - a;
            }
            report("fileput_zc_persistent.kernel", t);
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)((char *)dm + off), (uint4 *)((char *)duser), (long long)nv);
                CK(hipStreamSynchronize(s));
                t[r] = now_us() - a;
            }
            report("fileget_zc_persistent.kernel", t);
            // the same with SDMA H2D into HBM, then the kernel storing into the file
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                CK(hipMemcpyAsync(dbuf, user, bytes, hipMemcpyHostToDevice, s));
                hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)dbuf, (uint4 *)((char *)dm + off), (long long)nv);
                CK(hipStreamSynchronize(s));
                t[r] = now_us() - a;
            }
            report("fileput_sdma_zcstore_persistent", t);
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                hipLaunchKernelGGL(k_swap4_x4, dim3((unsigned)((nv + 1023) / 1024)), dim3(256), 0, s, (const uint4 *)((char *)dm + off), (uint4 *)dbuf, (long long)nv);
                CK(hipMemcpyAsync(user2, dbuf, bytes, hipMemcpyDeviceToHost, s));
                CK(hipStreamSynchronize(s));
                t[r] = now_us() - a;
            }
            report("fileget_zcx4load_sdma_persistent", t);
            CK(hipHostUnregister(m));
            munmap(m, span);
            // get per call: map + register + kernel (file pages -> user) + unregister + unmap
            CK(hipHostUnregister(user));
            CK(hipHostRegister(user2, bytes, hipHostRegisterMapped));
            void *duser2 = nullptr;
            CK(hipHostGetDevicePointer(&duser2, user2, 0));
            for (int r = 0; r < reps; r++) {
                double a = now_us();
                unsigned char *mm = (unsigned char *)mmap(NULL, span, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, base);
                if (mm == MAP_FAILED) return 2;
                if (hipHostRegister(mm, span, hipHostRegisterMapped | hipHostRegisterReadOnly) != hipSuccess) {
                    (void)hipGetLastError();
                    CK(hipHostRegister(mm, span, hipHostRegisterMapped));
                }
                void *dmm = nullptr;
                CK(hipHostGetDevicePointer(&dmm, mm, 0));
                hipLaunchKernelGGL(k_swap4, dim3(grid), dim3(256), 0, s, (const uint4 *)((char *)dmm + off), (uint4 *)duser2, (long long)nv);
                CK(hipStreamSynchronize(s));
                CK(hipHostUnregister(mm));
                munmap(mm, span);
                t[r] = now_us() - a;
            }
            report("fileget_zc.total(map+reg+kernel+unreg+unmap)", t);
            for (size_t i = 0; i < bytes / 4; i++)
                if (user2[i] != user[i]) { fprintf(stderr, "fileget mismatch at %zu\n", i); return 3; }
            printf("# fileget_zc verified\n");
            CK(hipHostUnregister(user2));
        } else {
            CK(hipHostUnregister(user));
        }
    }
    // the reference's sequences, for the same box
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        cpu_swap4(user, bytes / 4);
        if (pwrite(fd, user, bytes, off) != (ssize_t)bytes) return 2;
        cpu_swap4(user, bytes / 4);
        t[r] = now_us() - a;
    }
    report("reference_put_swap_pwrite_swap", t);
    for (int r = 0; r < reps; r++) {
        double a = now_us();
        if (pread(fd, user2, bytes, off) != (ssize_t)bytes) return 2;
        cpu_swap4(user2, bytes / 4);
        t[r] = now_us() - a;
    }
    report("reference_get_pread_swap", t);
    close(fd);
    unlink(path);
    printf("# ok\n");
    return 0;
}
