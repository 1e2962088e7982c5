// pncx_pairs.hpp -- the (xtype, itype) conversion matrix of
// ncmpii_putn_NC_<X>/ncmpii_getn_NC_<X> (convert_swap.m4:202-330):
// 10 numeric external types x 11 internal types.
#pragma once
#include "pncx_kern.hpp"

#define PNCX_ROW(M, XT)                                                          \
    M(XT, PNCX_ITYPE_SCHAR) M(XT, PNCX_ITYPE_UCHAR) M(XT, PNCX_ITYPE_SHORT)      \
    M(XT, PNCX_ITYPE_USHORT) M(XT, PNCX_ITYPE_INT) M(XT, PNCX_ITYPE_UINT)        \
    M(XT, PNCX_ITYPE_LONG) M(XT, PNCX_ITYPE_FLOAT) M(XT, PNCX_ITYPE_DOUBLE)      \
    M(XT, PNCX_ITYPE_LONGLONG) M(XT, PNCX_ITYPE_ULONGLONG)
#define PNCX_ALL_PAIRS(M)                                                        \
    PNCX_ROW(M, NC_BYTE) PNCX_ROW(M, NC_UBYTE) PNCX_ROW(M, NC_SHORT)             \
    PNCX_ROW(M, NC_USHORT) PNCX_ROW(M, NC_INT) PNCX_ROW(M, NC_UINT)              \
    PNCX_ROW(M, NC_FLOAT) PNCX_ROW(M, NC_DOUBLE) PNCX_ROW(M, NC_INT64)           \
    PNCX_ROW(M, NC_UINT64)

namespace pncx {
// same representation: routed to the swap/copy kernels by the host code
template <int XT, int IT>
struct same_rep {
    static constexpr bool value =
        (XT == NC_BYTE && IT == PNCX_ITYPE_SCHAR) || (XT == NC_UBYTE && IT == PNCX_ITYPE_UCHAR) ||
        (XT == NC_SHORT && IT == PNCX_ITYPE_SHORT) || (XT == NC_USHORT && IT == PNCX_ITYPE_USHORT) ||
        (XT == NC_INT && IT == PNCX_ITYPE_INT) || (XT == NC_UINT && IT == PNCX_ITYPE_UINT) ||
        (XT == NC_FLOAT && IT == PNCX_ITYPE_FLOAT) || (XT == NC_DOUBLE && IT == PNCX_ITYPE_DOUBLE) ||
        (XT == NC_INT64 && (IT == PNCX_ITYPE_LONGLONG || IT == PNCX_ITYPE_LONG)) ||
        (XT == NC_UINT64 && IT == PNCX_ITYPE_ULONGLONG);
};
}  // namespace pncx
