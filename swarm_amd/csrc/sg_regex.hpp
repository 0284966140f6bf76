// sg_regex.hpp — regex signatures -> set of byte-class DFAs (host side).
//
// Dialect: Python `re` on bytes patterns (the oracle: re.search existence), subset:
//   literals and escaped metacharacters, '.', classes [...] / [^...] with ranges and
//   \d \w \s \D \W \S inside, escapes \t \n \r \f \v \xHH \0, anchors ^ $ \A \Z,
//   groups ( ) (?: ) (?P<name> ), alternation |, quantifiers * + ? {n} {n,} {,m} {n,m}
//   and their lazy forms (same existence semantics), global (?i) and scoped (?i:...).
//   word boundaries \b \B (ASCII word bytes [0-9A-Za-z_]).
// Rejected with SG_E_UNSUPPORTED: backreferences, lookaround, other inline flags.
// Search semantics: a pattern matches a record if some substring matches; '^'/'\A' hold
// at offset 0 only, '$'/'\Z' at the record end only (records hold no '\n').
#pragma once
#include <stdint.h>
#include <vector>

namespace sg {

struct RegexDFA {
    uint32_t n_states = 0, n_classes = 0;  // state 0 = dead, 1 = start; class n_classes-1 = EOL
    uint8_t cls[256];
    uint32_t eol_class = 0;
    std::vector<uint32_t> delta;    // n_states * n_classes
    std::vector<uint32_t> acc_off;  // n_states + 1
    std::vector<uint32_t> acc_ids;  // pattern ids accepted on entering a state
    // Anchored DFA (no restart at every byte): a match is searched by running it from
    // every start offset. State 1 starts at the record start; a start at offset p > 0 uses
    // mid_start[word(byte p-1)]. Built for a prefiltered pattern whose search DFA exceeds
    // the state budget (a counted repeat overlapping its own restarts, e.g. <[^>]{1,512}).
    bool anchored = false;
    uint32_t mid_start[2] = {0, 0};
};

// Builds DFAs for all patterns, splitting the set so that no DFA exceeds the state budget.
int regex_build_set(const uint8_t *pats, const uint32_t *offs, uint32_t n, uint32_t flags,
                    std::vector<RegexDFA> *out);

// Prefiltered plan (Hyperscan-style). Every pattern with a literal factor set F (any match
// contains one string of F, compared case-insensitively, every string >= 3 bytes) is
// "filtered": a case-insensitive Aho-Corasick pass over all factor strings proposes
// (record, pattern) candidates, each verified by that pattern's own DFA. The remaining
// patterns are scanned by the multi-pattern DFA groups.
struct RegexPlan {
    std::vector<RegexDFA> groups;              // unfiltered patterns
    std::vector<std::vector<uint8_t>> factors; // distinct lowercase factor strings
    std::vector<uint32_t> fac_off, fac_pids;   // factor -> patterns (CSR)
    std::vector<RegexDFA> singles;             // one DFA per filtered pattern
    std::vector<uint32_t> single_pid;          // pattern id of singles[k]
    std::vector<uint32_t> single_of_pid;       // pattern id -> index into singles (or ~0)
};
int regex_build_plan(const uint8_t *pats, const uint32_t *offs, uint32_t n, uint32_t flags,
                     RegexPlan *plan);
// Parse-only check for one pattern (SG_OK or SG_E_UNSUPPORTED/SG_E_INVAL).
int regex_check(const uint8_t *pat, uint32_t len, uint32_t flags);

}  // namespace sg
