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
// SG_STAGE=0: the dedup gathers records from the input in every pass after the sort instead
// of staging them once in sorted order (sg_dedup.hip k_stage; A/B and the tests' second path).
inline bool sw_stage() { return env_switch("SG_STAGE", false); }
// SG_FUSED_DIFF=1: the new-record diff inside the unique emit (k_emit_uniq_diff) instead of
// its own pass over the unique output (k_diff_tile). Off: measured 534 us for the fused emit
// against 438 for emit + split + diff + new-record count on C2.
inline bool sw_fused_diff() { return env_switch("SG_FUSED_DIFF", false); }
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

}  // namespace sg
