// sg_switches.hpp — the library's ONLY environment reads: test switches that force an
// alternative engine which is exact on its own, so the parity tests can compare both paths
// on the same inputs. None changes results; none is a tuning knob (those were removed in
// round 3 with their losing pipelines, tools/experiments/). Each is read once per process.
#pragma once
#include <stdlib.h>

namespace sg {

inline bool env_switch(const char *name, bool dflt) {
    const char *v = getenv(name);
    return v ? atoi(v) != 0 : dflt;
}

// SG_FORCE_LITFILTER=1: literal matchers use the hashed q-gram filter even when the
// Aho-Corasick automaton fits the LDS hot table (tests/test_gpu_match.py, test_gpu_fused.py).
inline bool sw_force_litfilter() { return env_switch("SG_FORCE_LITFILTER", false); }
// SG_DFA_MULTI=0: factor-less regex groups walked one launch per automaton instead of the
// packed multi-automaton kernel (tests/test_gpu_match.py).
inline bool sw_dfa_multi() { return env_switch("SG_DFA_MULTI", true); }
// SG_HIT_RADIX=1: (record, signature) hits sorted by the LSD radix sort instead of the
// record-bucket LDS sort (tests/test_gpu_match.py).
inline bool sw_hit_radix() { return env_switch("SG_HIT_RADIX", false); }
// SG_REGEX_ANCHORED=1: every prefiltered regex verified by its anchored DFA
// (tests/test_gpu_match.py).
inline bool sw_regex_anchored() { return env_switch("SG_REGEX_ANCHORED", false); }
// SG_LIT_SCHEME=0|1: literal filters run the two-class (0) or the joint (1) class scheme
// instead of timing both on the first large input (tests/test_gpu_match.py).
inline int sw_lit_scheme() {
    const char *v = getenv("SG_LIT_SCHEME");
    return v ? (atoi(v) != 0 ? 1 : 0) : -1;
}
// The dedup's all-segments mode (sg_dedup.hip SEG_ALL_UNIQ): SG_SEG_ALL=0 never, 1 (default)
// by the context's last unique fraction, 2 always (tests).
inline int sw_seg_all() {
    const char *v = getenv("SG_SEG_ALL");
    return v ? atoi(v) : 1;
}
// SG_LIT_TRIAL_LOG=1: print the literal filter's scheme trial counts (calibration).
inline bool sw_lit_trial_log() { return env_switch("SG_LIT_TRIAL_LOG", false); }
// SG_TM_SORT=1: nuclei templates evaluated through the sort path instead of the
// record-wave evaluator (tests/test_gpu_templates.py).
inline bool sw_tm_sort() { return env_switch("SG_TM_SORT", false); }

// SG_SYNC_CHECK=1 (diagnosis only): every kernel launch is followed by a stream sync, so an
// asynchronous fault is reported with the name of the kernel that raised it.
inline bool sw_sync_check() {
    static const bool on = env_switch("SG_SYNC_CHECK", false);
    return on;
}

}  // namespace sg
