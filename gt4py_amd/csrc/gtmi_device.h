// gtmi_device.h -- device-side helpers shared by every generated gt:mi355x stencil.
//
// Numerics follow the reference numpy backend (gtc/ufuncs.py + numpy's own loops):
//  * min/max propagate NaN like np.minimum / np.maximum,
//  * mod is np.remainder (npy_divmod: result takes the sign of the divisor),
//  * round is np.round (half to even = rint), round_away_from_zero is
//    copysign(floor(|x| + 0.5), x) (gtc/ufuncs.py:31-33),
//  * integer power / remainder follow numpy's integer loops.
// Everything is compiled with -ffp-contract=off so no FMA contraction changes rounding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GTMI_DEV __device__ __forceinline__

// host side: a data-dimension index clamped into [0, n) (no out-of-bounds component pointer)
static inline int64_t gtmi_clamp_index(int64_t x, int64_t n) { return x < 0 ? 0 : (x >= n ? n - 1 : x); }

namespace gtmi {

// ---------------------------------------------------------------- wave shuffles (wave64)
// Value of `v` held by lane (lane_id + delta) mod 64. Executed by all lanes of the wave
// (callers hoist shuffles out of divergent control flow).
GTMI_DEV double shfl(double v, int delta) {
    const int src = (int)(__lane_id() + delta) & 63;
    return __shfl(v, src, 64);
}
GTMI_DEV float shfl(float v, int delta) {
    const int src = (int)(__lane_id() + delta) & 63;
    return __shfl(v, src, 64);
}
GTMI_DEV int64_t shfl(int64_t v, int delta) {
    const int src = (int)(__lane_id() + delta) & 63;
    return (int64_t)__shfl((long long)v, src, 64);
}
GTMI_DEV int32_t shfl(int32_t v, int delta) {
    const int src = (int)(__lane_id() + delta) & 63;
    return __shfl((int)v, src, 64);
}
GTMI_DEV int16_t shfl(int16_t v, int delta) { return (int16_t)shfl((int32_t)v, delta); }
GTMI_DEV int8_t shfl(int8_t v, int delta) { return (int8_t)shfl((int32_t)v, delta); }
GTMI_DEV bool shfl(bool v, int delta) { return shfl((int32_t)v, delta) != 0; }

// Compile-time delta: |delta| == 1 is a DPP wave rotate (v_mov_b32_dpp wave_rol:1 / wave_ror:1,
// a VALU move with no LDS-crossbar round trip); other deltas fall back to ds_bpermute. Same
// result as shfl(v, delta): lane l receives the value of lane (l + delta) mod 64.
template <int D> GTMI_DEV int32_t dpp_rot32(int32_t v) {
    static_assert(D == 1 || D == -1, "DPP wave rotate by one lane only");
    return __builtin_amdgcn_update_dpp(0, v, D == 1 ? 0x134 : 0x13C, 0xf, 0xf, false);
}
template <int D, typename T> GTMI_DEV T shfl_c(T v) {
    if constexpr (D == 1 || D == -1) {
        if constexpr (sizeof(T) == 8) {
            int64_t x;
            __builtin_memcpy(&x, &v, 8);
            const int32_t lo = dpp_rot32<D>((int32_t)(x & 0xffffffff));
            const int32_t hi = dpp_rot32<D>((int32_t)(x >> 32));
            const int64_t y = (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
            T r;
            __builtin_memcpy(&r, &y, 8);
            return r;
        } else if constexpr (sizeof(T) == 4) {
            int32_t x;
            __builtin_memcpy(&x, &v, 4);
            const int32_t y = dpp_rot32<D>(x);
            T r;
            __builtin_memcpy(&r, &y, 4);
            return r;
        } else {
            return shfl(v, D);
        }
    } else {
        return shfl(v, D);
    }
}

// ---------------------------------------------------------------- clamps
GTMI_DEV int clampi(int x, int lo, int hi) { return x < lo ? lo : (x > hi ? hi : x); }

// ---------------------------------------------------------------- math (numpy semantics)
template <typename T> GTMI_DEV bool isnan_(T) { return false; }
template <> GTMI_DEV bool isnan_<double>(double x) { return __builtin_isnan(x); }
template <> GTMI_DEV bool isnan_<float>(float x) { return __builtin_isnan(x); }

template <typename T> GTMI_DEV T minimum(T a, T b) {
    if (isnan_(a)) return a;
    if (isnan_(b)) return b;
    return a < b ? a : b;
}
template <typename T> GTMI_DEV T maximum(T a, T b) {
    if (isnan_(a)) return a;
    if (isnan_(b)) return b;
    return a > b ? a : b;
}

GTMI_DEV double absolute(double x) { return fabs(x); }
GTMI_DEV float absolute(float x) { return fabsf(x); }
GTMI_DEV int64_t absolute(int64_t x) { return x < 0 ? -x : x; }
GTMI_DEV int32_t absolute(int32_t x) { return x < 0 ? -x : x; }
GTMI_DEV int16_t absolute(int16_t x) { return (int16_t)(x < 0 ? -x : x); }
GTMI_DEV int8_t absolute(int8_t x) { return (int8_t)(x < 0 ? -x : x); }
GTMI_DEV bool absolute(bool x) { return x; }

GTMI_DEV double remainder_(double a, double b) {
    double mod = fmod(a, b);
    if (b == 0.0) return mod;
    if (mod != 0.0) {
        if ((b < 0) != (mod < 0)) mod += b;
    } else {
        mod = copysign(0.0, b);
    }
    return mod;
}
GTMI_DEV float remainder_(float a, float b) {
    float mod = fmodf(a, b);
    if (b == 0.0f) return mod;
    if (mod != 0.0f) {
        if ((b < 0) != (mod < 0)) mod += b;
    } else {
        mod = copysignf(0.0f, b);
    }
    return mod;
}
template <typename T> GTMI_DEV T remainder_int(T a, T b) {
    if (b == 0) return 0;
    T r = a % b;
    if (r != 0 && ((r < 0) != (b < 0))) r += b;
    return r;
}
GTMI_DEV int64_t remainder_(int64_t a, int64_t b) { return remainder_int(a, b); }
GTMI_DEV int32_t remainder_(int32_t a, int32_t b) { return remainder_int(a, b); }
GTMI_DEV int16_t remainder_(int16_t a, int16_t b) { return remainder_int(a, b); }
GTMI_DEV int8_t remainder_(int8_t a, int8_t b) { return remainder_int(a, b); }

template <typename T> GTMI_DEV T square(T x) { return x * x; }

template <typename T> GTMI_DEV T ipow(T base, T exp) {
    if (exp < 0) return (T)0;  // numpy raises; keep it defined on device
    T r = 1;
    while (exp) {
        if (exp & 1) r *= base;
        base *= base;
        exp >>= 1;
    }
    return r;
}

GTMI_DEV double round_half_even(double x) { return rint(x); }
GTMI_DEV float round_half_even(float x) { return rintf(x); }
GTMI_DEV double round_away(double x) { return copysign(floor(fabs(x) + 0.5), x); }
GTMI_DEV float round_away(float x) { return copysignf(floorf(fabsf(x) + 0.5f), x); }

}  // namespace gtmi

namespace gtmi {
// V contiguous elements of T, aligned to their size: one global_load/store of V*sizeof(T) bytes.
template <typename T, int V> struct alignas(sizeof(T) * V) vec {
    T v[V];
};
}  // namespace gtmi

// Runtime switch GTMI_VECTOR=1 forces the scalar (V=1) plane kernels (host side, read once).
#include <stdlib.h>
static inline int gtmi_env_vector(void) {
    static int v = -1;
    if (v < 0) {
        const char* s = getenv("GTMI_VECTOR");
        v = s ? atoi(s) : 0;
    }
    return v;
}

// Multiplier a with gcd(a, n) == 1 near n / golden ratio: w -> (w * a) mod n scatters work
// items bijectively (host side).
static inline int gtmi_coprime_multiplier(long long n) {
    if (n <= 2) return 1;
    long long a = (long long)(n * 0.6180339887) | 1;
    for (;; a += 2) {
        long long x = a, y = n;
        while (y) { long long t = x % y; x = y; y = t; }
        if (x == 1) return (int)(a % n);
    }
}

namespace gtmi {
// 16-B-per-lane memory ops on clang ext vectors (bool/int8/int16 use the struct path).
template <typename T, int V> using evec = T __attribute__((ext_vector_type(V)));

template <typename T, int V, bool NT> GTMI_DEV void vload(const T* p, T (&out)[V]) {
    const evec<T, V>* q = reinterpret_cast<const evec<T, V>*>(p);
    evec<T, V> x;
    if constexpr (NT) x = __builtin_nontemporal_load(q); else x = *q;
#pragma unroll
    for (int e = 0; e < V; ++e) out[e] = x[e];
}
template <typename T, int V, bool NT> GTMI_DEV void vstore(T* p, const T (&in)[V]) {
    evec<T, V> x;
#pragma unroll
    for (int e = 0; e < V; ++e) x[e] = in[e];
    evec<T, V>* q = reinterpret_cast<evec<T, V>*>(p);
    if constexpr (NT) __builtin_nontemporal_store(x, q); else *q = x;
}
// Buffer descriptor of one row: `nbytes` valid bytes from `row` (0 = the row is skipped: every
// load through it returns 0 without a memory access). Built from wave-uniform values only.
GTMI_DEV __amdgpu_buffer_rsrc_t row_rsrc(const void* row, int32_t nbytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(row), (short)0, nbytes, 0x00020000);
}
// V elements (8 or 16 bytes) at byte offset `off` of a row descriptor; NT = non-temporal
template <typename T, int V, bool NT> GTMI_DEV void bload(__amdgpu_buffer_rsrc_t rs, int32_t off, T (&out)[V]) {
    static_assert(sizeof(T) * V == 16 || sizeof(T) * V == 8, "bload moves 8 or 16 bytes");
    if constexpr (sizeof(T) * V == 16) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, NT ? 2 : 0);
        __builtin_memcpy(out, &x, 16);
    } else {
        const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, NT ? 2 : 0);
        __builtin_memcpy(out, &x, 8);
    }
}
// V elements (8 or 16 bytes) to byte offset `off` of a row descriptor (dropped when out of range)
template <typename T, int V, bool NT> GTMI_DEV void bstore(__amdgpu_buffer_rsrc_t rs, int32_t off, const T (&in)[V]) {
    static_assert(sizeof(T) * V == 16 || sizeof(T) * V == 8, "bstore moves 8 or 16 bytes");
    if constexpr (sizeof(T) * V == 16) {
        using W = decltype(__builtin_amdgcn_raw_buffer_load_b128(rs, 0, 0, 0));
        W x;
        __builtin_memcpy(&x, in, 16);
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, off, 0, NT ? 2 : 0);
    } else {
        using W = decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0));
        W x;
        __builtin_memcpy(&x, in, 8);
        __builtin_amdgcn_raw_buffer_store_b64(x, rs, off, 0, NT ? 2 : 0);
    }
}
template <typename T, bool NT> GTMI_DEV T sload(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}
template <typename T, bool NT> GTMI_DEV void sstore(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}
}  // namespace gtmi

namespace gtmi {
// Workgroup barrier for LDS exchange only: waits for this wave's LDS operations, then s_barrier.
// Loads and stores to global memory stay in flight across it (__syncthreads() would also drain
// them with vmcnt(0)); the "memory" clobber keeps the compiler from moving LDS accesses across.
GTMI_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
}  // namespace gtmi
