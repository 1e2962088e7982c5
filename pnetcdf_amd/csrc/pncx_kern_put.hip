// pncx_kern_put.hip -- PUT kernels: internal -> external (XDR big-endian),
// one instance per (xtype, itype) of ncmpix_putn_NC_<X>_<itype>
// (ncx.m4 NCX_PUTN :2620-2704 / NCX_PUTN_BYTE :2561-2581), plus the
// fillp == NULL variants of the codecs that then keep or swap the bytes
// already in xbuf.
#include "pncx_pairs.hpp"

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

extern "C" int pncxk_put(int xtype, int itype, int preserve, const pncxk_args *a) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return put_one<XT, IT>(preserve, a);
        PNCX_ALL_PAIRS(CASE)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

extern "C" int pncxk_batch_put(int xtype, int itype, int preserve, const pncxk_batch_args *a) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return put_batch<XT, IT>(preserve, a);
        PNCX_ALL_PAIRS(CASE)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

extern "C" int pncxk_batch_fused_put(int xtype, int itype, int preserve, const pncxk_batch_args *a,
                                     const pncxk_batch_args *m) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return put_fused<XT, IT>(preserve, a, m);
        PNCX_ALL_PAIRS(CASE)
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

extern "C" int pncxk_imap_put(int xtype, int itype, int preserve, const pncxk_args *a, const pncxk_imap *m) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return put_imap<XT, IT>(preserve, a, m);
        PNCX_ALL_PAIRS(CASE)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

extern "C" int pncxk_opinfo_get_get(int xtype, int itype, pncxk_opinfo *o);

extern "C" int pncxk_opinfo_getput(int kind, int xtype, int itype, int preserve, pncxk_opinfo *o) {
    (void)preserve;
    if (kind == PNCXK_GET) return pncxk_opinfo_get_get(xtype, itype, o);
    if (kind != PNCXK_PUT) return NC_EINVAL;
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return put_info<XT, IT>(o);
        PNCX_ALL_PAIRS(CASE)
#undef CASE
        default: return NC_EBADTYPE;
    }
}
