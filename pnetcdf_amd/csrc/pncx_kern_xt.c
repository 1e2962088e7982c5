/*
 * pncx_kern_xt.c -- the conversion launchers by external type.
 *
 * pncx_kern_put.hip and pncx_kern_get.hip are compiled once per external
 * type (Makefile, -DPNCX_XT), so that each type's kernels form a code object
 * of their own: HIP loads a code object on a device at the first launch from
 * it, and one object holding all 220 conversions' ~6900 kernels took 180 ms
 * to load against ~18 ms for one type's (profiles/r05p_first_launch.txt).
 * These are the entry points the rest of the library calls (pncx_shim.h,
 * pncx_kern_swap.hip), switching on the external type as
 * ncmpii_putn_NC_<X>/ncmpii_getn_NC_<X> do (convert_swap.m4:202-330).
 */
#include "pncx.h"
#include "pncx_shim.h"

/* the external types of the matrix (pncx_pairs.hpp PNCX_ALL_PAIRS) */
#define PNCX_XTS(M) M(1) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11)

#define DECL(X)                                                                                        \
    int pncxk_put_x##X(int, int, int, const pncxk_args *);                                             \
    int pncxk_batch_put_x##X(int, int, int, const pncxk_batch_args *);                                 \
    int pncxk_batch_fused_put_x##X(int, int, int, const pncxk_batch_args *, const pncxk_batch_args *); \
    int pncxk_imap_put_x##X(int, int, int, const pncxk_args *, const pncxk_imap *);                    \
    int pncxk_opinfo_put_x##X(int, int, pncxk_opinfo *);                                               \
    int pncxk_get_x##X(int, int, const pncxk_args *);                                                  \
    int pncxk_batch_get_x##X(int, int, const pncxk_batch_args *);                                      \
    int pncxk_batch_fused_get_x##X(int, int, const pncxk_batch_args *, const pncxk_batch_args *);      \
    int pncxk_imap_get_x##X(int, int, const pncxk_args *, const pncxk_imap *);                         \
    int pncxk_opinfo_get_get_x##X(int, int, pncxk_opinfo *);                                          \
    int pncxk_load_put_x##X(void);                                                                     \
    int pncxk_load_get_x##X(void);
PNCX_XTS(DECL)
#undef DECL

/* declared for the HIP files in pncx_kern_swap.hip */
int pncxk_batch_put(int xtype, int itype, int preserve, const pncxk_batch_args *a);
int pncxk_batch_get(int xtype, int itype, const pncxk_batch_args *a);
int pncxk_batch_fused_put(int xtype, int itype, int preserve, const pncxk_batch_args *a, const pncxk_batch_args *m);
int pncxk_batch_fused_get(int xtype, int itype, const pncxk_batch_args *a, const pncxk_batch_args *m);
int pncxk_imap_put(int xtype, int itype, int preserve, const pncxk_args *a, const pncxk_imap *m);
int pncxk_imap_get(int xtype, int itype, const pncxk_args *a, const pncxk_imap *m);
int pncxk_opinfo_getput(int kind, int xtype, int itype, int preserve, pncxk_opinfo *o);

#define SWITCH(CALL)                        \
    switch (xtype) {                        \
        PNCX_XTS(CALL)                      \
        default: return NC_EBADTYPE;        \
    }

int pncxk_put(int xtype, int itype, int preserve, const pncxk_args *a)
{
#define C(X) case X: return pncxk_put_x##X(xtype, itype, preserve, a);
    SWITCH(C)
#undef C
}

int pncxk_batch_put(int xtype, int itype, int preserve, const pncxk_batch_args *a)
{
#define C(X) case X: return pncxk_batch_put_x##X(xtype, itype, preserve, a);
    SWITCH(C)
#undef C
}

int pncxk_batch_fused_put(int xtype, int itype, int preserve, const pncxk_batch_args *a, const pncxk_batch_args *m)
{
#define C(X) case X: return pncxk_batch_fused_put_x##X(xtype, itype, preserve, a, m);
    SWITCH(C)
#undef C
}

int pncxk_imap_put(int xtype, int itype, int preserve, const pncxk_args *a, const pncxk_imap *m)
{
#define C(X) case X: return pncxk_imap_put_x##X(xtype, itype, preserve, a, m);
    SWITCH(C)
#undef C
}

int pncxk_get(int xtype, int itype, const pncxk_args *a)
{
#define C(X) case X: return pncxk_get_x##X(xtype, itype, a);
    SWITCH(C)
#undef C
}

int pncxk_batch_get(int xtype, int itype, const pncxk_batch_args *a)
{
#define C(X) case X: return pncxk_batch_get_x##X(xtype, itype, a);
    SWITCH(C)
#undef C
}

int pncxk_batch_fused_get(int xtype, int itype, const pncxk_batch_args *a, const pncxk_batch_args *m)
{
#define C(X) case X: return pncxk_batch_fused_get_x##X(xtype, itype, a, m);
    SWITCH(C)
#undef C
}

int pncxk_imap_get(int xtype, int itype, const pncxk_args *a, const pncxk_imap *m)
{
#define C(X) case X: return pncxk_imap_get_x##X(xtype, itype, a, m);
    SWITCH(C)
#undef C
}

int pncxk_opinfo_getput(int kind, int xtype, int itype, int preserve, pncxk_opinfo *o)
{
    (void)preserve;
    if (kind == PNCXK_GET) {
#define C(X) case X: return pncxk_opinfo_get_get_x##X(xtype, itype, o);
        SWITCH(C)
#undef C
    }
    if (kind != PNCXK_PUT) return NC_EINVAL;
#define C(X) case X: return pncxk_opinfo_put_x##X(xtype, itype, o);
    SWITCH(C)
#undef C
}

/* load the put and get code objects of one external type on the current
 * device (pncx_preload_xtypes) */
int pncxk_load_xtype(int xtype)
{
#define C(X) case X: { const int e = pncxk_load_put_x##X(); return e ? e : pncxk_load_get_x##X(); }
    SWITCH(C)
#undef C
}
