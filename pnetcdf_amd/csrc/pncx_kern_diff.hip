// pncx_kern_diff.hip -- first-difference search of two HBM arrays, the data
// comparison of ncmpidiff (src/utils/ncmpidiff/ncmpidiff_core.c:200-236,
// CHECK_VAR_DIFF).  Both variables are read through the conversion path into
// HBM as their native type; this kernel finds the smallest index where they
// differ, either exactly (b1 != b2) or beyond both tolerances:
//     diff = |(promoted) b1 - b2|, ratio = diff / max(ABS(b1), ABS(b2)),
//     a difference when !(diff <= tol_diff || ratio <= tol_ratio)
// with the reference's C arithmetic: the subtraction and ABS() happen in the
// promoted type (int for 1/2-byte types, wrapping for int/uint/int64/uint64,
// float for float) before the conversion to double.  HBM-bound: both arrays
// are streamed once with 16-byte nontemporal loads; a hit is an atomicMin on
// a 64-bit index.
#include "pncx_kern.hpp"

using namespace pncx;

namespace {

template <typename T> struct Promo { using type = T; };
template <> struct Promo<signed char> { using type = int; };
template <> struct Promo<unsigned char> { using type = int; };
template <> struct Promo<short> { using type = int; };
template <> struct Promo<unsigned short> { using type = int; };

// x - y and -x in the promoted type, wrapping like x86-64 integer arithmetic
template <typename P>
__device__ __forceinline__ P sub_wrap(P x, P y) {
    if constexpr (std::is_integral<P>::value) {
        using U = typename std::make_unsigned<P>::type;
        return (P)((U)x - (U)y);
    } else {
        return x - y;
    }
}
template <typename P>
__device__ __forceinline__ P neg_wrap(P x) {
    if constexpr (std::is_integral<P>::value) {
        using U = typename std::make_unsigned<P>::type;
        return (P)((U)0 - (U)x);
    } else {
        return -x;
    }
}

template <typename T, bool TOL>
__device__ __forceinline__ bool differs(T a, T b, double td, double tr) {
    if constexpr (!TOL) {
        return !(a == b);
    } else {
        using P = typename Promo<T>::type;
        if (a == b) return false;
        const P pa = (P)a, pb = (P)b;
        // ABS(x) ((x) >= 0) ? (x) : (-x);  UABS(x) (x)  (ncmpidiff_core.c:200-201)
        const double abs_a = std::is_unsigned<T>::value ? (double)pa : (double)(pa >= 0 ? pa : neg_wrap(pa));
        const double abs_b = std::is_unsigned<T>::value ? (double)pb : (double)(pb >= 0 ? pb : neg_wrap(pb));
        const double abs_max = abs_a > abs_b ? abs_a : abs_b;
        double diff = (double)sub_wrap(pa, pb);
        diff = diff >= 0 ? diff : -diff;
        const double ratio = diff / abs_max;
        return !(diff <= td || ratio <= tr);
    }
}

template <typename T, bool TOL>
__global__ __launch_bounds__(256) void k_first_diff(const uint8_t *a, const uint8_t *b, int64_t head, int64_t nvec,
                                                    int64_t n, double td, double tr, unsigned long long *first) {
    constexpr int V = 16 / sizeof(T);
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t best = n;
    for (int64_t v = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x; v < nvec; v += stride) {
        const int64_t e0 = head + v * V;
        const u32x4 va = ld16<true>(a + e0 * sizeof(T)), vb = ld16<true>(b + e0 * sizeof(T));
        T ea[V], eb[V];
        __builtin_memcpy(ea, &va, 16);
        __builtin_memcpy(eb, &vb, 16);
#pragma unroll
        for (int i = V - 1; i >= 0; i--)
            if (differs<T, TOL>(ea[i], eb[i], td, tr)) best = e0 + i;
        if (best < n) break;                     // later vectors of this lane are larger
    }
    if (blockIdx.x == 0) {                       // unaligned head and the tail
        for (int64_t e = threadIdx.x; e < head; e += 256)
            if (e < best && differs<T, TOL>(ld_unaligned<T>(a + e * sizeof(T)), ld_unaligned<T>(b + e * sizeof(T)), td, tr))
                best = e;
        for (int64_t e = head + nvec * V + threadIdx.x; e < n; e += 256)
            if (e < best && differs<T, TOL>(ld_unaligned<T>(a + e * sizeof(T)), ld_unaligned<T>(b + e * sizeof(T)), td, tr))
                best = e;
    }
    if (best < n) atomicMin(first, (unsigned long long)best);
}

template <typename T>
int launch(const void *a, const void *b, int64_t n, int tol, double td, double tr, unsigned long long *first,
           hipStream_t st) {
    const uintptr_t pa = (uintptr_t)a, pb = (uintptr_t)b;
    int64_t head = -1;
    for (int64_t h = 0; h < 16 && h <= n; h++)
        if (((pa + h * sizeof(T)) & 15) == 0 && ((pb + h * sizeof(T)) & 15) == 0) { head = h; break; }
    int64_t nvec = 0;
    if (head < 0) head = n;                      // no common alignment: all scalar (block 0)
    else nvec = (n - head) / (16 / (int64_t)sizeof(T));
    const int grid = launch_grid(nvec > 0 ? nvec : 1, 1);
    if (tol) hipLaunchKernelGGL((k_first_diff<T, true>), dim3(grid), dim3(256), 0, st, (const uint8_t *)a,
                                (const uint8_t *)b, head, nvec, n, td, tr, first);
    else hipLaunchKernelGGL((k_first_diff<T, false>), dim3(grid), dim3(256), 0, st, (const uint8_t *)a,
                            (const uint8_t *)b, head, nvec, n, td, tr, first);
    return hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE;
}

}  // namespace

// itype: PNCX_ITYPE_* (text compares as signed char, as ncmpi_get_vara_text_all's char)
extern "C" int pncxk_first_diff(const void *a, const void *b, long long n, int itype, int tol, double td,
                                double tr, unsigned long long *first, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (n <= 0) return 0;
    switch (itype) {
        case PNCX_ITYPE_SCHAR: case PNCX_ITYPE_CHAR: return launch<signed char>(a, b, n, tol, td, tr, first, st);
        case PNCX_ITYPE_UCHAR: return launch<unsigned char>(a, b, n, tol, td, tr, first, st);
        case PNCX_ITYPE_SHORT: return launch<short>(a, b, n, tol, td, tr, first, st);
        case PNCX_ITYPE_USHORT: return launch<unsigned short>(a, b, n, tol, td, tr, first, st);
        case PNCX_ITYPE_INT: return launch<int>(a, b, n, tol, td, tr, first, st);
        case PNCX_ITYPE_UINT: return launch<unsigned>(a, b, n, tol, td, tr, first, st);
        case PNCX_ITYPE_FLOAT: return launch<float>(a, b, n, tol, td, tr, first, st);
        case PNCX_ITYPE_DOUBLE: return launch<double>(a, b, n, tol, td, tr, first, st);
        case PNCX_ITYPE_LONG: case PNCX_ITYPE_LONGLONG: return launch<long long>(a, b, n, tol, td, tr, first, st);
        case PNCX_ITYPE_ULONGLONG: return launch<unsigned long long>(a, b, n, tol, td, tr, first, st);
        default: return NC_EBADTYPE;
    }
}
