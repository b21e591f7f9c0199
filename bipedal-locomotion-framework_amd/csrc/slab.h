// slab.h — coalesced staging of row-major slabs between HBM and LDS.
//
// The per-item kernels (one lane per contact / system / polygon / spline query) keep their
// inputs and outputs item-major: item q owns a row of W doubles.  Read or written lane-by-lane,
// such a row is a W*8-byte stride between the lanes of a wave.  The loads then touch 64 lines
// per instruction, and the stores write partial lines (read-modify-write in the memory side:
// 1.5-3x the algorithmic bytes, profiles/r01_stream_*).  Instead, a workgroup moves its whole slab
// (`rows` consecutive items) with consecutive lanes on consecutive doubles, 16 B per lane when
// the slab is contiguous and aligned, and the lanes then read or write their own row in LDS.
// LDS rows are padded to an odd stride SW so the per-lane row accesses do not conflict.
//
// U loads per lane are issued before the first LDS write, so a workgroup keeps U * NT * 8 (or
// 16) bytes in flight.  A loop that loads one element and stores it to LDS before issuing the
// next load serialises on HBM latency (the first version of dcm_rollout_kernel: 0.65 ms, 20 %
// of the HBM roofline).
#pragma once
#ifndef BLF_NT_STORE
#define BLF_NT_STORE 1
#endif

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace blf {

// A 16-B store of a streamed output (written once, not re-read by the kernel): non-temporal, so
// the output stream does not displace the inputs from the caches (the write-dominated quintic
// evaluation: 0.773 -> 0.731 ms; reads and the other kernels unchanged).  BLF_NT_STORE=0: plain.
__device__ __forceinline__ void st_stream(double2* p, double2 v)
{
#if BLF_NT_STORE
    typedef double d2v __attribute__((ext_vector_type(2)));
    d2v w;
    w.x = v.x;
    w.y = v.y;
    __builtin_nontemporal_store(w, reinterpret_cast<d2v*>(p));
#else
    *p = v;
#endif
}

// The same for 8-B / 4-B streamed outputs (phase expansion's offsets and facet counts).
__device__ __forceinline__ void st_stream(double* p, double v)
{
#if BLF_NT_STORE
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

__device__ __forceinline__ void st_stream(int32_t* p, int32_t v)
{
#if BLF_NT_STORE
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// A streamed output stored non-temporally (NT) or plainly, chosen per launch by the output's size.
template <bool NT, class T>
__device__ __forceinline__ void st_out(T* p, T v)
{
    if constexpr (NT) st_stream(p, v);
    else *p = v;
}

// Element e of a slab with W columns is row e / W.  (e + 0.5) / W lies at least 0.5 / W from an
// integer; in float the product's error is below 2^-22 * rows, so the row is exact for
// rows * W < 2^20 and W < 2^10 (all slabs here: rows <= 256, W <= 64).
struct SlabIdx {
    float inv;
    int W;
    __device__ __forceinline__ explicit SlabIdx(int w) : inv(1.0f / (float)w), W(w) {}
    __device__ __forceinline__ int row(int e) const { return (int)(((float)e + 0.5f) * inv); }
};

__device__ __forceinline__ int odd_stride(int w) { return w | 1; }

// s[r * SW + c] = g[r * GS + c] for r < rows, c < W.
template <int NT, int U>
__device__ __forceinline__ void slab_load(double* __restrict__ s, int SW,
                                          const double* __restrict__ g, int64_t GS, int rows,
                                          int W)
{
    const int t = threadIdx.x;
    const int n = rows * W;
    const SlabIdx ix(W);
    if (GS == W && ((uintptr_t)g & 15) == 0) {
        const double2* g2 = reinterpret_cast<const double2*>(g);
        const int n2 = n >> 1;
        for (int base = 0; base < n2; base += U * NT) {
            double2 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = base + u * NT + t;
                if (j < n2) v[u] = g2[j];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = base + u * NT + t;
                if (j < n2) {
                    const int e = 2 * j;
                    const int r0 = ix.row(e), r1 = ix.row(e + 1);
                    s[r0 * SW + (e - r0 * W)] = v[u].x;
                    s[r1 * SW + (e + 1 - r1 * W)] = v[u].y;
                }
            }
        }
        if ((n & 1) && t == 0) {
            const int e = n - 1, r = ix.row(e);
            s[r * SW + (e - r * W)] = g[e];
        }
        return;
    }
    for (int base = 0; base < n; base += U * NT) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = base + u * NT + t;
            if (e < n) {
                const int r = ix.row(e);
                v[u] = g[(int64_t)r * GS + (e - r * W)];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = base + u * NT + t;
            if (e < n) {
                const int r = ix.row(e);
                s[r * SW + (e - r * W)] = v[u];
            }
        }
    }
}

// g[r * GS + c] = s[r * SW + c] for r < rows, c < W.
template <int NT, int U>
__device__ __forceinline__ void slab_store(double* __restrict__ g, int64_t GS,
                                           const double* __restrict__ s, int SW, int rows, int W)
{
    const int t = threadIdx.x;
    const int n = rows * W;
    const SlabIdx ix(W);
    if (GS == W && ((uintptr_t)g & 15) == 0) {
        double2* g2 = reinterpret_cast<double2*>(g);
        const int n2 = n >> 1;
        if (SW == W && ((uintptr_t)s & 15) == 0) {
            // unpadded rows (odd W): the LDS slab is the global slab, 16-B LDS reads with no row
            // arithmetic (the quintic evaluation's 9-double rows: two float row divisions, two
            // address computations and two 8-B LDS reads per 16-B store before)
            const double2* s2 = reinterpret_cast<const double2*>(s);
            for (int base = 0; base < n2; base += U * NT) {
                double2 v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int j = base + u * NT + t;
                    if (j < n2) v[u] = s2[j];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int j = base + u * NT + t;
                    if (j < n2) st_stream(g2 + j, v[u]);
                }
            }
            if ((n & 1) && t == 0) g[n - 1] = s[n - 1];
            return;
        }
        for (int base = 0; base < n2; base += U * NT) {
            double2 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = base + u * NT + t;
                if (j < n2) {
                    const int e = 2 * j;
                    const int r0 = ix.row(e), r1 = ix.row(e + 1);
                    v[u].x = s[r0 * SW + (e - r0 * W)];
                    v[u].y = s[r1 * SW + (e + 1 - r1 * W)];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = base + u * NT + t;
                if (j < n2) st_stream(g2 + j, v[u]);
            }
        }
        if ((n & 1) && t == 0) {
            const int e = n - 1, r = ix.row(e);
            g[e] = s[r * SW + (e - r * W)];
        }
        return;
    }
    for (int base = 0; base < n; base += U * NT) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = base + u * NT + t;
            if (e < n) {
                const int r = ix.row(e);
                v[u] = s[r * SW + (e - r * W)];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = base + u * NT + t;
            if (e < n) {
                const int r = ix.row(e);
                g[(int64_t)r * GS + (e - r * W)] = v[u];
            }
        }
    }
}

// dst[i] = src[i] for i < n: a workgroup's contiguous slab copied without LDS.  The stores are
// nontemporal (written once, never re-read here); a plain copy loop is also rewritten into a
// memcpy call by the compiler, which costs scratch.
template <int NT, int U>
__device__ __forceinline__ void slab_copy(double* __restrict__ dst, const double* __restrict__ src,
                                          int n)
{
    const int t = threadIdx.x;
    if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
        const double2* s2 = reinterpret_cast<const double2*>(src);
        double2* d2 = reinterpret_cast<double2*>(dst);
        const int n2 = n >> 1;
        for (int base = 0; base < n2; base += U * NT) {
            double2 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = base + u * NT + t;
                if (j < n2) v[u] = s2[j];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = base + u * NT + t;
                if (j < n2) {
                    __builtin_nontemporal_store(v[u].x, &d2[j].x);
                    __builtin_nontemporal_store(v[u].y, &d2[j].y);
                }
            }
        }
        if ((n & 1) && t == 0) __builtin_nontemporal_store(src[n - 1], dst + n - 1);
        return;
    }
    for (int base = 0; base < n; base += U * NT) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = base + u * NT + t;
            if (e < n) v[u] = src[e];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = base + u * NT + t;
            if (e < n) __builtin_nontemporal_store(v[u], dst + e);
        }
    }
}

}  // namespace blf
