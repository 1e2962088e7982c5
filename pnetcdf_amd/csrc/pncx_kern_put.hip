// pncx_kern_put.hip -- PUT kernels: internal -> external (XDR big-endian),
// one instance per (xtype, itype) of ncmpix_putn_NC_<X>_<itype>
// (ncx.m4 NCX_PUTN :2620-2704 / NCX_PUTN_BYTE :2561-2581), plus the
// fillp == NULL variants of the codecs that then keep or swap the bytes
// already in xbuf.
#include "pncx_pairs.hpp"

// Compiled once per external type (-DPNCX_XT=<NC_* value>, Makefile): each
// type's kernels are a code object of their own, which HIP loads on a device
// at the first launch from it -- ~18 ms for one type's instead of 180 ms for
// all ten (profiles/r05p_first_launch.txt).  pncx_kern_xt.c dispatches on
// the external type.
#ifndef PNCX_XT
#error "compile with -DPNCX_XT=<external type>"
#endif
#define PNCX_FN2(name, x) name##_x##x
#define PNCX_FN1(name, x) PNCX_FN2(name, x)
#define PNCX_FN(name) PNCX_FN1(name, PNCX_XT)

using namespace pncx;

namespace {
template <int XT, int IT>
int put_one(int preserve, const pncxk_args *a) {
    if constexpr (same_rep<XT, IT>::value) {
        return NC_EINVAL;
    } else {
        if constexpr (null_fill_preserves<XT, IT>::value)
            if (preserve) return launch_stream<PutOp<XT, IT, true>>(a);
        return launch_stream<PutOp<XT, IT, false>>(a);
    }
}
template <int XT, int IT>
int put_batch(int preserve, const pncxk_batch_args *a) {
    if constexpr (same_rep<XT, IT>::value) {
        return NC_EINVAL;
    } else {
        if constexpr (null_fill_preserves<XT, IT>::value)
            if (preserve) return launch_batch<PutOp<XT, IT, true>>(a);
        return launch_batch<PutOp<XT, IT, false>>(a);
    }
}
template <int XT, int IT>
int put_fused(int preserve, const pncxk_batch_args *a, const pncxk_batch_args *m) {
    if constexpr (same_rep<XT, IT>::value) return NC_EINVAL;
    else if (preserve) return PNCXK_NOFUSE;
    else return launch_batch_fused<PutOp<XT, IT, false>>(a, m);
}
template <int XT, int IT>
int put_info(pncxk_opinfo *o) {
    OpInfo<PutOp<XT, IT, false>>::fill(o);
    return 0;
}
}  // namespace

#define PNCX_KEY(XT, IT) ((XT) * 16 + (IT))

extern "C" int PNCX_FN(pncxk_put)(int xtype, int itype, int preserve, const pncxk_args *a) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return put_one<XT, IT>(preserve, a);
        PNCX_ROW(CASE, PNCX_XT)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

extern "C" int PNCX_FN(pncxk_batch_put)(int xtype, int itype, int preserve, const pncxk_batch_args *a) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return put_batch<XT, IT>(preserve, a);
        PNCX_ROW(CASE, PNCX_XT)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

extern "C" int PNCX_FN(pncxk_batch_fused_put)(int xtype, int itype, int preserve, const pncxk_batch_args *a,
                                     const pncxk_batch_args *m) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return put_fused<XT, IT>(preserve, a, m);
        PNCX_ROW(CASE, PNCX_XT)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

namespace {
template <int XT, int IT>
int put_imap(int preserve, const pncxk_args *a, const pncxk_imap *m) {
    if constexpr (same_rep<XT, IT>::value) {
        return NC_EINVAL;
    } else {
        if constexpr (null_fill_preserves<XT, IT>::value)
            if (preserve) return launch_imap<PutOp<XT, IT, true>>(a, m, 1);
        return launch_imap<PutOp<XT, IT, false>>(a, m, 1);
    }
}
}  // namespace

extern "C" int PNCX_FN(pncxk_imap_put)(int xtype, int itype, int preserve, const pncxk_args *a, const pncxk_imap *m) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return put_imap<XT, IT>(preserve, a, m);
        PNCX_ROW(CASE, PNCX_XT)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

extern "C" int PNCX_FN(pncxk_opinfo_put)(int xtype, int itype, pncxk_opinfo *o) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return put_info<XT, IT>(o);
        PNCX_ROW(CASE, PNCX_XT)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

// A kernel of this file's code object, launched never: a function-attribute
// query on it makes HIP load the object on the current device, which
// pncx_preload_xtypes does at enddef for the types a file defines
// (pncx_nc.c), off the first data call.
__global__ void PNCX_FN(k_put_object)() {}
extern "C" int PNCX_FN(pncxk_load_put)(void) {
    hipFuncAttributes fa;
    return hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&PNCX_FN(k_put_object))) == hipSuccess
               ? 0 : PNCX_EDEVICE;
}
