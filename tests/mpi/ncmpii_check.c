/*
 * ncmpii_check.c -- drives the reference-named, MPI-typed conversion entry
 * points of libpncx_ncmpii.so (include/pncx_ncmpii.h; the reference's
 * src/drivers/include/common.h:147-221) with real MPI_Datatype handles.
 * Test infrastructure: tests/test_gpu_c_api.py writes the cases, runs this
 * program and compares every output with the CPU oracle.
 *
 *   ncmpii_check run <cases.bin> <out.bin>
 *
 * cases.bin: records of little-endian int64 fields
 *   op (0 putn, 1 getn, 2 in_swapn, 3 need_convert), cdf, xtype, mpi,
 *   nelems (for in_swapn: esize in xtype), has_fill, fill (8 raw bytes),
 *   nbytes, then nbytes of input: putn = ibuf then the initial xbuf,
 *   getn = xbuf, in_swapn = the buffer.
 * out.bin: per record, int64 status, int64 nbytes, then the output bytes
 *   (putn: xbuf, getn: ibuf, in_swapn: the buffer, need_convert: none).
 * mpi: index into MPI_TYPES below; the last two are types the conversion
 * has no itype for (NC_EBADTYPE, convert_swap.m4:245,311).
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pncx_ncmpii.h"

static MPI_Datatype mpi_type(int i)
{
    switch (i) {
    case 0: return MPI_SIGNED_CHAR;
    case 1: return MPI_UNSIGNED_CHAR;
    case 2: return MPI_SHORT;
    case 3: return MPI_UNSIGNED_SHORT;
    case 4: return MPI_INT;
    case 5: return MPI_UNSIGNED;
    case 6: return MPI_LONG;
    case 7: return MPI_FLOAT;
    case 8: return MPI_DOUBLE;
    case 9: return MPI_LONG_LONG_INT;
    case 10: return MPI_UNSIGNED_LONG_LONG;
    case 11: return MPI_CHAR;
    case 12: return MPI_BYTE;          /* not a conversion itype */
    default: return MPI_LONG_DOUBLE;   /* not a conversion itype */
    }
}

static int mpi_size(int i)
{
    static const int sz[] = {1, 1, 2, 2, 4, 4, 8, 4, 8, 8, 8, 1, 1, 16};
    return sz[i < 13 ? i : 13];
}

static int xsize(int xtype)
{
    switch (xtype) {
    case NC_BYTE: case NC_CHAR: case NC_UBYTE: return 1;
    case NC_SHORT: case NC_USHORT: return 2;
    case NC_INT: case NC_UINT: case NC_FLOAT: return 4;
    default: return 8;
    }
}

static int putn(int cdf, int xtype, void *x, const void *b, MPI_Offset n, MPI_Datatype t, void *fill)
{
    switch (xtype) {
    case NC_BYTE: return ncmpii_putn_NC_BYTE(cdf, x, b, n, t, fill);
    case NC_CHAR: return ncmpii_putn_NC_CHAR(x, b, n, t);
    case NC_SHORT: return ncmpii_putn_NC_SHORT(x, b, n, t, fill);
    case NC_INT: return ncmpii_putn_NC_INT(x, b, n, t, fill);
    case NC_FLOAT: return ncmpii_putn_NC_FLOAT(x, b, n, t, fill);
    case NC_DOUBLE: return ncmpii_putn_NC_DOUBLE(x, b, n, t, fill);
    case NC_UBYTE: return ncmpii_putn_NC_UBYTE(x, b, n, t, fill);
    case NC_USHORT: return ncmpii_putn_NC_USHORT(x, b, n, t, fill);
    case NC_UINT: return ncmpii_putn_NC_UINT(x, b, n, t, fill);
    case NC_INT64: return ncmpii_putn_NC_INT64(x, b, n, t, fill);
    case NC_UINT64: return ncmpii_putn_NC_UINT64(x, b, n, t, fill);
    default: return NC_EBADTYPE;
    }
}

static int getn(int cdf, int xtype, const void *x, void *b, MPI_Offset n, MPI_Datatype t)
{
    switch (xtype) {
    case NC_BYTE: return ncmpii_getn_NC_BYTE(cdf, x, b, n, t);
    case NC_CHAR: return ncmpii_getn_NC_CHAR(x, b, n, t);
    case NC_SHORT: return ncmpii_getn_NC_SHORT(x, b, n, t);
    case NC_INT: return ncmpii_getn_NC_INT(x, b, n, t);
    case NC_FLOAT: return ncmpii_getn_NC_FLOAT(x, b, n, t);
    case NC_DOUBLE: return ncmpii_getn_NC_DOUBLE(x, b, n, t);
    case NC_UBYTE: return ncmpii_getn_NC_UBYTE(x, b, n, t);
    case NC_USHORT: return ncmpii_getn_NC_USHORT(x, b, n, t);
    case NC_UINT: return ncmpii_getn_NC_UINT(x, b, n, t);
    case NC_INT64: return ncmpii_getn_NC_INT64(x, b, n, t);
    case NC_UINT64: return ncmpii_getn_NC_UINT64(x, b, n, t);
    default: return NC_EBADTYPE;
    }
}

static int64_t rd(FILE *f)
{
    int64_t v;
    if (fread(&v, 8, 1, f) != 1) return INT64_MIN;
    return v;
}

static void wr(FILE *f, int64_t v) { fwrite(&v, 8, 1, f); }

int main(int argc, char **argv)
{
    FILE *in, *out;
    int ncase = 0;
    MPI_Init(&argc, &argv);
    if (argc != 4 || strcmp(argv[1], "run") != 0) {
        fprintf(stderr, "usage: %s run <cases.bin> <out.bin>\n", argv[0]);
        MPI_Finalize();
        return 2;
    }
    in = fopen(argv[2], "rb");
    out = fopen(argv[3], "wb");
    if (in == NULL || out == NULL) { perror("open"); MPI_Finalize(); return 2; }
    for (;;) {
        const int64_t op = rd(in);
        int64_t cdf, xtype, mi, n, has_fill, nbytes, st = 0;
        uint8_t fill[8], *b;
        if (op == INT64_MIN) break;
        cdf = rd(in);
        xtype = rd(in);
        mi = rd(in);
        n = rd(in);
        has_fill = rd(in);
        if (fread(fill, 1, 8, in) != 8) break;
        nbytes = rd(in);
        b = (uint8_t *)malloc((size_t)nbytes + 16);
        if (b == NULL || (nbytes > 0 && fread(b, 1, (size_t)nbytes, in) != (size_t)nbytes)) {
            fprintf(stderr, "short case %d\n", ncase);
            MPI_Finalize();
            return 2;
        }
        if (op == 0) {                          /* putn: ibuf | xinit -> xbuf */
            const int64_t ib = n * mpi_size((int)mi);
            uint8_t *x = b + ib;                /* the initial xbuf, converted in place */
            st = putn((int)cdf, (int)xtype, x, b, n, mpi_type((int)mi), has_fill ? fill : NULL);
            wr(out, st);
            wr(out, n * xsize((int)xtype));
            fwrite(x, 1, (size_t)(n * xsize((int)xtype)), out);
        } else if (op == 1) {                   /* getn: xbuf -> ibuf */
            const int64_t ib = n * mpi_size((int)mi);
            uint8_t *o = (uint8_t *)calloc((size_t)ib + 16, 1);
            st = getn((int)cdf, (int)xtype, b, o, n, mpi_type((int)mi));
            wr(out, st);
            wr(out, ib);
            fwrite(o, 1, (size_t)ib, out);
            free(o);
        } else if (op == 2) {                   /* in_swapn: esize in xtype */
            ncmpii_in_swapn(b, n, (int)xtype);
            wr(out, 0);
            wr(out, nbytes);
            fwrite(b, 1, (size_t)nbytes, out);
        } else {                                /* need_convert */
            st = ncmpii_need_convert((int)cdf, (int)xtype, mpi_type((int)mi));
            wr(out, st);
            wr(out, 0);
        }
        free(b);
        ncase++;
    }
    fclose(in);
    fclose(out);
    printf("cases %d\n", ncase);
    MPI_Finalize();
    return 0;
}
