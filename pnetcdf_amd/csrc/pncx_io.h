/*
 * pncx_io.h -- parallel POSIX I/O for the file layer (internal).
 *
 * A fixed pool of threads copies between staging memory and the file with
 * pread/pwrite.  A job is a list of file runs (offset, length, memory); it
 * is split into byte ranges of about equal size, one per thread, so a single
 * large run and many small runs both spread over the pool.  Jobs are
 * asynchronous: the data path converts chunk k+1 on the GPU while the pool
 * writes chunk k (pncx_nc.c).
 */
#ifndef PNCX_IO_H
#define PNCX_IO_H

#include <pthread.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pio_run {
    long long off, len;
    unsigned char *mem;
} pio_run;

typedef struct pio_batch {
    pthread_mutex_t m;
    pthread_cond_t c;
    int pending;
    int err;
} pio_batch;

void pio_batch_init(pio_batch *b);
void pio_batch_destroy(pio_batch *b);
/* Queue runs[0..n) (copied); returns immediately.  Small jobs run inline. */
int  pio_submit(pio_batch *b, int fd, int write, const pio_run *runs, size_t n);
/* Wait for every job submitted on b; returns the first error (NC_EWRITE/NC_EREAD). */
int  pio_wait(pio_batch *b);
/* The job on the calling thread with pread/pwrite (no pool, no mapping). */
int  pio_rw_inline(int fd, int write, const pio_run *runs, size_t n);
/* Synchronous convenience: submit + wait. */
int  pio_rw(int fd, int write, const pio_run *runs, size_t n);
int  pio_threads(void);
/* A read job split over up to `parts` pool threads whatever its size
 * (pieces of at least 64 KiB): the inline gets' chunks (pncx_nc.c). */
int  pio_read_split(pio_batch *b, int fd, const pio_run *runs, size_t n, int parts);


int  pio_write_all(int fd, const void *buf, size_t n, long long off);
int  pio_read_all(int fd, void *buf, size_t n, long long off);

#ifdef __cplusplus
}
#endif
#endif
