// sg_route.hpp — byte-range routing of records by byte-string splitters (the multi-GPU
// exchange and the C5 local parts): shared by the routing kernels of sg_abi.hip and the
// parse-and-route pass of sg_lines.hip (k_lines_route).
//
// Byte-string splitters (SG_SPLIT_BYTES = 64 bytes each at most): part(record) = number of
// splitters <= record in bytewise order (shorter-is-smaller). Unlike a key0 splitter, a
// byte splitter can fall inside a run of records sharing their first 7 bytes (https://...,
// 10.0.x.y:port), so range parts stay balanced on URL and IP data. Both sides are compared
// as 8 big-endian words of their first 64 bytes (zero past the end), then by length: words
// differ => the first differing word decides; all equal => one is a prefix of the other
// within 64 bytes (or they are equal there) and the longer one is larger, which is exact
// because a splitter never has more than 64 bytes.
#pragma once
#include "sg_common.hpp"

namespace sg {

constexpr uint32_t SPL_W = 64, SPL_WORDS = SPL_W / 8;

__device__ __forceinline__ void head_words(const uint8_t *__restrict__ buf, uint32_t s, uint32_t e,
                                           uint64_t (&w)[SPL_WORDS]) {
    const uint32_t len = e - s;
#pragma unroll
    for (uint32_t k = 0; k < SPL_WORDS; ++k) {
        const uint32_t o = 8u * k;
        w[k] = o < len ? load_le(buf, s + o, min(len - o, 8u)) : 0ull;
    }
}

// record < splitter (BE words)
__device__ __forceinline__ bool head_less(const uint64_t (&w)[SPL_WORDS], uint32_t len, const uint64_t *sw,
                                          uint32_t slen) {
    int r = 0;
#pragma unroll
    for (uint32_t k = 0; k < SPL_WORDS; ++k) {
        if (r == 0) {
            const uint64_t a = w[k], b = sw[k];
            if (a != b) r = a < b ? -1 : 1;
        }
    }
    return r ? r < 0 : len < slen;
}

// Splitter q's key0 (its first 7 bytes + min(len, 8)), from its packed BE words.
__device__ __forceinline__ uint64_t split_key0(const uint64_t *split_w, const uint32_t *split_len, uint32_t q) {
    const uint32_t l = split_len[q];
    return (split_w[q * SPL_WORDS] & ~0xffull) | (uint64_t)(l < 8u ? l : 8u);
}

// The part of the record [s, e) with key0 rk: binary search over the ns splitter key0s
// (s_k0); a tie on a full tag compares the first 64 bytes (head_less; words and lengths from
// split_w / split_len). e may be unknown (~0u): then the record's length is found by a
// '\n' search over at most SPL_W + 1 bytes (a longer record compares as longer than any
// splitter with the same 64 bytes), bytes at or past n read as the end.
__device__ __forceinline__ uint32_t route_record(const uint8_t *__restrict__ buf, uint64_t n, uint32_t s, uint32_t e,
                                                 uint64_t rk, const uint64_t *s_k0, uint32_t ns,
                                                 const uint64_t *__restrict__ split_w,
                                                 const uint32_t *__restrict__ split_len) {
    uint64_t w[SPL_WORDS];
    bool loaded = false;
    uint32_t lo = 0, hi = ns;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint64_t sk = s_k0[mid];
        bool less;
        if (rk != sk) {
            less = rk < sk;
        } else if ((rk & 0xffu) < 8u) {
            less = false;  // the same record bytes: splitter <= record
        } else {
            if (!loaded) {
                if (e == ~0u) {
                    uint32_t l = 0;
                    while (l <= SPL_W && (uint64_t)s + l < n && buf[s + l] != 0x0a) ++l;
                    e = s + l;
                }
                head_words(buf, s, e, w);
#pragma unroll
                for (uint32_t k = 0; k < SPL_WORDS; ++k) w[k] = __builtin_bswap64(w[k]);
                loaded = true;
            }
            less = head_less(w, e - s, split_w + mid * SPL_WORDS, split_len[mid]);
        }
        if (!less) lo = mid + 1; else hi = mid;
    }
    return lo;
}

}  // namespace sg
