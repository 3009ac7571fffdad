// Host-side word checks of the in-order commit (Resolver::resolve_mask in
// kbg_session.cpp): the host mirror's verdict on the 64 nodes of one candidate
// word at once, for words holding many candidates touched since their scan.
// Built by the host compiler only (kbg_walk.cpp: AVX-512 behind a run-time
// CPU check); the mirror rows are the session's AoS Res rows (3 doubles).
#pragma once
#include <stdint.h>

namespace kbg {

// true when this CPU runs the AVX-512 word checks (else callers walk node by node)
bool walk_simd();

// Nodes [n0, n0 + cnt) (cnt <= 64) against request r (3 doubles) with the
// per-dimension tolerances mins (Resource.LessEqual, resource_info.go:142-146;
// the same IEEE operations as res_le, so the verdicts are identical): bit j of
// *fi = node n0+j fits in Idle, of *fr = it does not but fits in Releasing;
// with cap, only nodes below their pod cap (nt < mt, predicates.go:125-127).
void word_fits(const double* idle, const double* rel, const int32_t* nt, const int32_t* mt, bool cap, const double* r,
               const double* mins, int32_t n0, int32_t cnt, uint64_t* fi, uint64_t* fr);

// bit j = mark[n0 + j] > base (the node was touched after the scan at `base`)
uint64_t word_newer(const int32_t* mark, int32_t n0, int32_t cnt, int32_t base);

// bit j = flags[n0 + j] != 0
uint64_t word_flags(const char* flags, int32_t n0, int32_t cnt);

}  // namespace kbg
