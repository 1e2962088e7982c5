// pncx_kern_get.hip -- GET kernels: external (XDR big-endian) -> internal,
// one instance per (xtype, itype) of ncmpix_getn_NC_<X>_<itype>
// (ncx.m4 NCX_GETN :2429-2495 / NCX_GETN_BYTE :2369-2392).
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
int get_one(const pncxk_args *a) {
    if constexpr (same_rep<XT, IT>::value) return NC_EINVAL;
    else return launch_stream<GetOp<XT, IT>>(a);
}
template <int XT, int IT>
int get_batch(const pncxk_batch_args *a) {
    if constexpr (same_rep<XT, IT>::value) return NC_EINVAL;
    else return launch_batch<GetOp<XT, IT>>(a);
}
template <int XT, int IT>
int get_fused(const pncxk_batch_args *a, const pncxk_batch_args *m) {
    if constexpr (same_rep<XT, IT>::value) return NC_EINVAL;
    else return launch_batch_fused<GetOp<XT, IT>>(a, m);
}
template <int XT, int IT>
int get_info(pncxk_opinfo *o) {
    OpInfo<GetOp<XT, IT>>::fill(o);
    return 0;
}
}  // namespace

#define PNCX_KEY(XT, IT) ((XT) * 16 + (IT))

extern "C" int PNCX_FN(pncxk_get)(int xtype, int itype, const pncxk_args *a) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return get_one<XT, IT>(a);
        PNCX_ROW(CASE, PNCX_XT)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

extern "C" int PNCX_FN(pncxk_batch_get)(int xtype, int itype, const pncxk_batch_args *a) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return get_batch<XT, IT>(a);
        PNCX_ROW(CASE, PNCX_XT)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

extern "C" int PNCX_FN(pncxk_batch_fused_get)(int xtype, int itype, const pncxk_batch_args *a, const pncxk_batch_args *m) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return get_fused<XT, IT>(a, m);
        PNCX_ROW(CASE, PNCX_XT)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

namespace {
template <int XT, int IT>
int get_imap(const pncxk_args *a, const pncxk_imap *m) {
    if constexpr (same_rep<XT, IT>::value) return NC_EINVAL;
    else return launch_imap<GetOp<XT, IT>>(a, m, 0);
}
}  // namespace

extern "C" int PNCX_FN(pncxk_imap_get)(int xtype, int itype, const pncxk_args *a, const pncxk_imap *m) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return get_imap<XT, IT>(a, m);
        PNCX_ROW(CASE, PNCX_XT)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

extern "C" int PNCX_FN(pncxk_opinfo_get_get)(int xtype, int itype, pncxk_opinfo *o) {
    switch (PNCX_KEY(xtype, itype)) {
#define CASE(XT, IT) case PNCX_KEY(XT, IT): return get_info<XT, IT>(o);
        PNCX_ROW(CASE, PNCX_XT)
#undef CASE
        default: return NC_EBADTYPE;
    }
}

// A kernel of this file's code object, launched never: a function-attribute
// query on it makes HIP load the object on the current device, which
// pncx_preload_xtypes does at enddef for the types a file defines
// (pncx_nc.c), off the first data call.
__global__ void PNCX_FN(k_get_object)() {}
extern "C" int PNCX_FN(pncxk_load_get)(void) {
    hipFuncAttributes fa;
    return hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&PNCX_FN(k_get_object))) == hipSuccess
               ? 0 : PNCX_EDEVICE;
}
