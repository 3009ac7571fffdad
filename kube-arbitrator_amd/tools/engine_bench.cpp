// Developer tool (not part of libkbgpu.so): times the host ordering engine of
// the allocate path alone, on a CPU-only machine. It includes the session
// source to reach the engine, runs open_session (which builds all host state
// and then stops at the missing device) and drives the predictor with every
// outcome = placed, i.e. the engine work of a cycle where everything fits.
#include "../csrc/kbg_session.cpp"

extern "C" double kbg_tool_engine_ns_per_step(const kbg_snapshot* snap, const kbg_options* o, int32_t reps,
                                              int64_t* steps_out, double* checksum, int32_t profile) {
  kbg::Session S;
  open_session(S, snap, o, nullptr);  // returns KBG_E_HIP on a machine without a device; host state is complete
  if (S.init.qlen == 0) return -1.0;
  double best = 1e30;
  int64_t steps = 0;
  uint64_t sum = 0;
  EngineProfile prof;
  for (int32_t r = 0; r < reps; ++r) {
    Engine E = S.init;
    prof = EngineProfile{};
    Ops ops{S, E, profile ? &prof : nullptr};
    steps = 0;
    sum = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const int32_t t = ops.next_task();
      if (t < 0) break;
      ops.apply(t, true);
      sum = (sum * 1000003u) ^ (uint64_t)t;  // order-sensitive
      ++steps;
    }
    const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
    best = std::min(best, ns / std::max<int64_t>(1, steps));
  }
  if (steps_out) *steps_out = steps;
  if (checksum) *checksum = (double)(sum >> 11);
  if (profile && prof.steps)
    fprintf(stderr, "cycles/step: qpop %.1f apply %.1f jfix %.1f qpush %.1f\n", (double)prof.qpop / prof.steps,
            (double)prof.apply / prof.steps, (double)prof.jtop / prof.steps, (double)prof.qpush / prof.steps);
  return best;
}

// Host side of kbg_session_update without a device: opens the snapshot's host
// state, applies the events to the inputs and re-derives; returns the node
// rows (Idle, Releasing, task count) and the pending candidates in job order,
// for comparison with a fresh snapshot of the updated cache (CPU test).
extern "C" int32_t kbg_tool_update_nodes(const kbg_snapshot* snap, const kbg_options* o, const kbg_event* ev,
                                         int32_t n, double* idle, double* rel, int32_t* ntasks, int32_t* pend,
                                         int32_t* n_pend) {
  kbg::Session S;
  if (ingest(S, snap, o) != KBG_OK) return -1;
  kbg::StaticHost sh;
  int outcome;
  if (derive_host(S, &sh, &outcome) != KBG_OK) return -2;
  S.n_classes = sh.n_classes;
  UpdateCtx U;
  U.seen.assign(S.n_nodes, 0);
  const auto t0 = std::chrono::steady_clock::now();
  for (int32_t i = 0; i < n; ++i)
    if (apply_event(S, U, ev[i]) != KBG_OK) return -3;
  const auto t1 = std::chrono::steady_clock::now();
  if (derive_host(S, nullptr, &outcome) != KBG_OK) return -4;
  if (getenv("KBG_TOOL_TIME"))
    fprintf(stderr, "[tool] %d events: apply %.3f ms, derive %.3f ms\n", n,
            std::chrono::duration<double, std::milli>(t1 - t0).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
  for (int32_t k = 0; k < S.n_nodes; ++k) {
    idle[3 * k] = S.idle[k].c;
    idle[3 * k + 1] = S.idle[k].m;
    idle[3 * k + 2] = S.idle[k].g;
    rel[3 * k] = S.rel[k].c;
    rel[3 * k + 1] = S.rel[k].m;
    rel[3 * k + 2] = S.rel[k].g;
    ntasks[k] = S.ntasks[k];
  }
  *n_pend = (int32_t)S.pend_all.size();
  std::copy(S.pend_all.begin(), S.pend_all.end(), pend);
  return outcome;
}
