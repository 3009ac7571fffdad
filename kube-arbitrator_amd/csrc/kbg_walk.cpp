// AVX-512 word checks of the in-order commit (kbg_walk.hpp). Host code only,
// compiled by the host compiler; every function carries its own target
// attribute and runs only after walk_simd() saw the CPU support it (the
// MI355X hosts' EPYC 9005 parts do). Masked loads never touch a node past
// n0 + cnt.
#include "kbg_walk.hpp"

#include <immintrin.h>

namespace kbg {

#define KBG_AVX512 __attribute__((target("avx512f,avx512dq,avx512vl,avx512bw")))

bool walk_simd() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
                         __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512bw");
  return ok;
}

namespace {

// res_le in one dimension: r < a || |a - r| < min
KBG_AVX512 inline __mmask8 le8(__m512d r, __m512d a, __m512d mn) {
  return _mm512_cmp_pd_mask(r, a, _CMP_LT_OQ) | _mm512_cmp_pd_mask(_mm512_abs_pd(_mm512_sub_pd(a, r)), mn, _CMP_LT_OQ);
}

// 8 AoS rows (c, m, g) = 24 doubles in 3 registers, each component collected
// by two two-source permutes; res_le of r against each row
KBG_AVX512 inline __mmask8 fits8(const double* p, uint32_t dmask, __m512d rc, __m512d rm, __m512d rg, __m512d mc,
                                 __m512d mm, __m512d mg) {
  const __m512i c1 = _mm512_setr_epi64(0, 3, 6, 9, 12, 15, 0, 0), c2 = _mm512_setr_epi64(0, 1, 2, 3, 4, 5, 10, 13);
  const __m512i m1 = _mm512_setr_epi64(1, 4, 7, 10, 13, 0, 0, 0), m2 = _mm512_setr_epi64(0, 1, 2, 3, 4, 8, 11, 14);
  const __m512i g1 = _mm512_setr_epi64(2, 5, 8, 11, 14, 0, 0, 0), g2 = _mm512_setr_epi64(0, 1, 2, 3, 4, 9, 12, 15);
  const __m512d z0 = _mm512_maskz_loadu_pd((__mmask8)dmask, p);
  const __m512d z1 = _mm512_maskz_loadu_pd((__mmask8)(dmask >> 8), p + 8);
  const __m512d z2 = _mm512_maskz_loadu_pd((__mmask8)(dmask >> 16), p + 16);
  const __m512d c = _mm512_permutex2var_pd(_mm512_permutex2var_pd(z0, c1, z1), c2, z2);
  const __m512d m = _mm512_permutex2var_pd(_mm512_permutex2var_pd(z0, m1, z1), m2, z2);
  const __m512d g = _mm512_permutex2var_pd(_mm512_permutex2var_pd(z0, g1, z1), g2, z2);
  return le8(rc, c, mc) & le8(rm, m, mm) & le8(rg, g, mg);
}

}  // namespace

KBG_AVX512 void word_fits(const double* idle, const double* rel, const int32_t* nt, const int32_t* mt, bool cap,
                          const double* r, const double* mins, int32_t n0, int32_t cnt, uint64_t* fi, uint64_t* fr) {
  const __m512d rc = _mm512_set1_pd(r[0]), rm = _mm512_set1_pd(r[1]), rg = _mm512_set1_pd(r[2]);
  const __m512d mc = _mm512_set1_pd(mins[0]), mm = _mm512_set1_pd(mins[1]), mg = _mm512_set1_pd(mins[2]);
  uint64_t oi = 0, orr = 0;
  for (int32_t j = 0; j < cnt; j += 8) {
    const int32_t n = n0 + j, left = cnt - j;
    const __mmask8 live = left >= 8 ? (__mmask8)0xff : (__mmask8)((1u << left) - 1);
    const uint32_t dmask = left >= 8 ? 0xffffffu : ((1u << (3 * left)) - 1);
    __mmask8 a = fits8(idle + 3 * (int64_t)n, dmask, rc, rm, rg, mc, mm, mg);
    __mmask8 b = fits8(rel + 3 * (int64_t)n, dmask, rc, rm, rg, mc, mm, mg);
    if (cap) {
      const __m256i vn = _mm256_maskz_loadu_epi32(live, nt + n), vm = _mm256_maskz_loadu_epi32(live, mt + n);
      const __mmask8 ok = _mm256_cmplt_epi32_mask(vn, vm);
      a &= ok;
      b &= ok;
    }
    a &= live;
    b &= (__mmask8)(live & ~a);
    oi |= (uint64_t)a << j;
    orr |= (uint64_t)b << j;
  }
  *fi = oi;
  *fr = orr;
}

KBG_AVX512 uint64_t word_newer(const int32_t* mark, int32_t n0, int32_t cnt, int32_t base) {
  const __m512i b = _mm512_set1_epi32(base);
  uint64_t out = 0;
  for (int32_t j = 0; j < cnt; j += 16) {
    const int32_t left = cnt - j;
    const __mmask16 live = left >= 16 ? (__mmask16)0xffff : (__mmask16)((1u << left) - 1);
    const __m512i v = _mm512_maskz_loadu_epi32(live, mark + n0 + j);
    out |= (uint64_t)(_mm512_cmpgt_epi32_mask(v, b) & live) << j;
  }
  return out;
}

KBG_AVX512 uint64_t word_flags(const char* flags, int32_t n0, int32_t cnt) {
  const __mmask64 live = cnt >= 64 ? ~0ull : ((1ull << cnt) - 1);
  const __m512i v = _mm512_maskz_loadu_epi8(live, flags + n0);
  return _mm512_test_epi8_mask(v, v) & live;
}

}  // namespace kbg
