// sg_regex.cpp — regex signatures -> byte-class DFAs for k_dfa_match (see sg_regex.hpp).
#include "sg_regex.hpp"
#include "sg_switches.hpp"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <bitset>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/swarmgpu.h"

namespace sg {
void set_error(const char *fmt, ...);

namespace {

using ByteSet = std::bitset<256>;

// ------------------------------------------------------------------ AST
struct Node {
    enum Kind { LIT, CAT, ALT, REP, BOL, EOL, WB, NWB, EMPTY } kind;
    ByteSet set;
    std::vector<std::unique_ptr<Node>> kids;
    int lo = 0, hi = -1;  // REP bounds, hi = -1: unbounded
};
using NodeP = std::unique_ptr<Node>;

static NodeP mk(Node::Kind k) {
    NodeP n(new Node());
    n->kind = k;
    return n;
}

struct ParseError {
    int code;
    const char *msg;
};

static ByteSet fold_set(const ByteSet &s) {
    ByteSet r = s;
    for (int c = 'a'; c <= 'z'; ++c)
        if (s[c] || s[c - 32]) { r.set(c); r.set(c - 32); }
    return r;
}

class Parser {
  public:
    Parser(const uint8_t *p, uint32_t n, bool nocase) : p_(p), n_(n), nocase_(nocase) {}
    NodeP parse() {
        // a global flag group (?aimsx) anywhere applies to the whole pattern (Python 3.10);
        // m and s are no-ops on records (no '\n' inside a record)
        for (uint32_t i = 0; i + 2 < n_; ++i) {
            if (p_[i] != '(' || p_[i + 1] != '?' || escaped(i)) continue;
            uint32_t j = i + 2;
            bool any = false, ic = false;
            while (j < n_ && flag_letter(p_[j])) { ic |= p_[j] == 'i'; ++j; any = true; }
            if (any && j < n_ && p_[j] == ')' && ic) nocase_ = true;
        }
        NodeP r = alt(nocase_);
        if (i_ != n_) throw ParseError{SG_E_INVAL, "unbalanced parenthesis"};
        return r;
    }

  private:
    const uint8_t *p_;
    uint32_t n_, i_ = 0;
    bool nocase_;
    int depth_ = 0;
    bool atom_grouped_ = false;  // the last atom was a parenthesized group

    static bool flag_letter(int c) { return c == 'a' || c == 'i' || c == 'm' || c == 's' || c == 'x' || c == 'L' || c == 'u'; }
    // (? flags ) or (? flags : ... ) starting at i_ (just after "(?"): returns 1 for a
    // global group, 2 for a scoped group (sets *ic), 0 if not a flag group.
    int flag_group(bool *ic) {
        uint32_t j = i_;
        bool any = false;
        *ic = false;
        while (j < n_ && flag_letter(p_[j])) {
            const int c = p_[j];
            if (c == 'x') throw ParseError{SG_E_UNSUPPORTED, "verbose flag (?x)"};
            if (c == 'L') throw ParseError{SG_E_UNSUPPORTED, "locale flag (?L)"};
            if (c == 'u') throw ParseError{SG_E_INVAL, "flag u with a bytes pattern"};
            *ic |= c == 'i';
            ++j;
            any = true;
        }
        if (!any || j >= n_) return 0;
        if (p_[j] == ')') { i_ = j + 1; return 1; }
        if (p_[j] == ':') { i_ = j + 1; return 2; }
        return 0;
    }
    bool escaped(uint32_t i) const {
        int bs = 0;
        while (i > 0 && p_[i - 1] == '\\') { ++bs; --i; }
        return bs & 1;
    }
    bool eof() const { return i_ >= n_; }
    int peek(uint32_t k = 0) const { return i_ + k < n_ ? p_[i_ + k] : -1; }

    NodeP alt(bool nc) {
        NodeP first = cat(nc);
        if (peek() != '|') return first;
        NodeP a = mk(Node::ALT);
        a->kids.push_back(std::move(first));
        while (peek() == '|') {
            ++i_;
            a->kids.push_back(cat(nc));
        }
        return a;
    }
    NodeP cat(bool nc) {
        NodeP c = mk(Node::CAT);
        while (!eof() && peek() != '|' && peek() != ')') c->kids.push_back(repeat(nc));
        if (c->kids.empty()) return mk(Node::EMPTY);
        if (c->kids.size() == 1) return std::move(c->kids[0]);
        return c;
    }
    bool quant_brace(int *lo, int *hi, uint32_t *len) {
        // {n} {n,} {,m} {n,m}; anything else is a literal '{'
        uint32_t j = i_ + 1;
        auto num = [&](int *v) {
            uint32_t s = j;
            long x = 0;
            while (j < n_ && p_[j] >= '0' && p_[j] <= '9') { x = x * 10 + (p_[j] - '0'); if (x > 100000) x = 100000; ++j; }
            *v = (int)x;
            return j > s;
        };
        int a = 0, b = -1;
        bool ha = num(&a);
        if (j < n_ && p_[j] == '}') {
            if (!ha) return false;
            *lo = a; *hi = a; *len = j + 1 - i_;
            return true;
        }
        if (j >= n_ || p_[j] != ',') return false;
        ++j;
        bool hb = num(&b);
        if (j >= n_ || p_[j] != '}') return false;
        *lo = ha ? a : 0;
        *hi = hb ? b : -1;
        *len = j + 1 - i_;
        return true;
    }
    NodeP repeat(bool nc) {
        NodeP atom_n = atom(nc);
        bool quantified = false;
        for (;;) {
            int c = peek();
            int lo, hi;
            uint32_t len = 1;
            if (c == '*') { lo = 0; hi = -1; }
            else if (c == '+') { lo = 1; hi = -1; }
            else if (c == '?') { lo = 0; hi = 1; }
            else if (c == '{') { if (!quant_brace(&lo, &hi, &len)) break; }
            else break;
            if (quantified) throw ParseError{SG_E_INVAL, "multiple repeat"};
            if (!quantified && (atom_n->kind == Node::EMPTY || atom_n->kind == Node::BOL || atom_n->kind == Node::EOL ||
                                atom_n->kind == Node::WB || atom_n->kind == Node::NWB) && !atom_grouped_)
                throw ParseError{SG_E_INVAL, "nothing to repeat"};
            if (hi >= 0 && hi < lo) throw ParseError{SG_E_INVAL, "min repeat greater than max repeat"};
            if (lo > 1000 || hi > 1000) throw ParseError{SG_E_UNSUPPORTED, "repeat bound above 1000"};
            i_ += len;
            if (peek() == '?') ++i_;  // lazy: same existence semantics
            NodeP r = mk(Node::REP);
            r->lo = lo;
            r->hi = hi;
            r->kids.push_back(std::move(atom_n));
            atom_n = std::move(r);
            quantified = true;
        }
        return atom_n;
    }
    NodeP lit(ByteSet s, bool nc) {
        NodeP n = mk(Node::LIT);
        n->set = nc ? fold_set(s) : s;
        return n;
    }
    static ByteSet digit() { ByteSet s; for (int c = '0'; c <= '9'; ++c) s.set(c); return s; }
    static ByteSet word() {
        ByteSet s = digit();
        for (int c = 'a'; c <= 'z'; ++c) { s.set(c); s.set(c - 32); }
        s.set('_');
        return s;
    }
    static ByteSet space() { ByteSet s; for (int c : {' ', '\t', '\n', '\r', '\f', '\v'}) s.set(c); return s; }
    int hexv(int c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }
    // escape after '\'; returns true with a set, or a single byte in *byte
    bool escape(bool in_class, ByteSet *set, int *byte, Node::Kind *anchor) {
        if (eof()) throw ParseError{SG_E_INVAL, "bad escape (end of pattern)"};
        int c = p_[i_++];
        *anchor = Node::EMPTY;
        switch (c) {
            case 'd': *set = digit(); return true;
            case 'D': *set = ~digit(); return true;
            case 'w': *set = word(); return true;
            case 'W': *set = ~word(); return true;
            case 's': *set = space(); return true;
            case 'S': *set = ~space(); return true;
            case 't': *byte = '\t'; return false;
            case 'n': *byte = '\n'; return false;
            case 'r': *byte = '\r'; return false;
            case 'f': *byte = '\f'; return false;
            case 'v': *byte = '\v'; return false;
            case 'a': *byte = 7; return false;
            case 'x': {
                int h1 = hexv(peek()), h2 = hexv(peek(1));
                if (h1 < 0 || h2 < 0) throw ParseError{SG_E_INVAL, "incomplete escape \\x"};
                i_ += 2;
                *byte = h1 * 16 + h2;
                return false;
            }
            case 'b':
                if (in_class) { *byte = 8; return false; }
                *anchor = Node::WB;
                return false;
            case 'B':
                if (in_class) throw ParseError{SG_E_INVAL, "bad escape \\B"};
                *anchor = Node::NWB;
                return false;
            case 'A':
                if (in_class) throw ParseError{SG_E_INVAL, "bad escape \\A"};
                *anchor = Node::BOL;
                return false;
            case 'Z':
                if (in_class) throw ParseError{SG_E_INVAL, "bad escape \\Z"};
                *anchor = Node::EOL;
                return false;
            default: break;
        }
        if (c >= '0' && c <= '7') {
            // \0, \0oo, or a 3-digit octal \ooo; \1..\9 otherwise are group references
            int v = c - '0';
            if (c == '0') {
                for (int k = 0; k < 2 && peek() >= '0' && peek() <= '7'; ++k) v = v * 8 + (p_[i_++] - '0');
                *byte = v;
                return false;
            }
            if (peek() >= '0' && peek() <= '7' && peek(1) >= '0' && peek(1) <= '7') {
                v = v * 64 + (p_[i_] - '0') * 8 + (p_[i_ + 1] - '0');
                i_ += 2;
                if (v > 255) throw ParseError{SG_E_INVAL, "octal escape out of range"};
                *byte = v;
                return false;
            }
            if (in_class) throw ParseError{SG_E_INVAL, "bad escape in class"};
            throw ParseError{SG_E_UNSUPPORTED, "backreference"};
        }
        if (c == '8' || c == '9') {
            if (in_class) throw ParseError{SG_E_INVAL, "bad escape in class"};
            throw ParseError{SG_E_UNSUPPORTED, "backreference"};
        }
        if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) throw ParseError{SG_E_INVAL, "bad escape"};
        *byte = c;
        return false;
    }
    NodeP klass(bool nc) {
        // after '['
        bool neg = false;
        if (peek() == '^') { neg = true; ++i_; }
        ByteSet s;
        bool first = true;
        for (;;) {
            if (eof()) throw ParseError{SG_E_INVAL, "unterminated character set"};
            int c = p_[i_];
            if (c == ']' && !first) { ++i_; break; }
            first = false;
            ++i_;
            int lo = -1;
            ByteSet es;
            if (c == '\\') {
                int b;
                Node::Kind an;
                if (escape(true, &es, &b, &an)) { s |= es; continue; }
                lo = b;
            } else {
                lo = c;
            }
            // range?
            if (peek() == '-' && peek(1) != ']' && peek(1) != -1) {
                ++i_;
                int hc = p_[i_++];
                int hi;
                if (hc == '\\') {
                    int b;
                    Node::Kind an;
                    if (escape(true, &es, &b, &an)) throw ParseError{SG_E_INVAL, "bad character range"};
                    hi = b;
                } else {
                    hi = hc;
                }
                if (hi < lo) throw ParseError{SG_E_INVAL, "bad character range"};
                for (int b = lo; b <= hi; ++b) s.set(b);
            } else {
                s.set(lo);
            }
        }
        if (nc) s = fold_set(s);
        if (neg) s = ~s;
        NodeP n = mk(Node::LIT);
        n->set = s;
        return n;
    }
    NodeP atom(bool nc) {
        int c = p_[i_];
        atom_grouped_ = false;
        if (c == '(') {
            ++i_;
            bool inner_nc = nc;
            if (peek() == '?') {
                ++i_;
                int d = peek();
                if (d == ':') { ++i_; }
                else if (d == 'P' && peek(1) == '<') {
                    i_ += 2;
                    while (!eof() && peek() != '>') ++i_;
                    if (eof()) throw ParseError{SG_E_INVAL, "unterminated group name"};
                    ++i_;
                } else if (flag_letter(d)) {
                    bool ic = false;
                    const int kind = flag_group(&ic);
                    if (kind == 1) return mk(Node::EMPTY);  // global flags, applied in parse()
                    if (kind == 0) throw ParseError{SG_E_UNSUPPORTED, "inline flag or extension"};
                    inner_nc = nc || ic;
                } else if (d == 'P' && peek(1) == '=') {
                    throw ParseError{SG_E_UNSUPPORTED, "named backreference"};
                } else if (d == '=' || d == '!' || d == '<') {
                    throw ParseError{SG_E_UNSUPPORTED, "lookaround"};
                } else {
                    throw ParseError{SG_E_UNSUPPORTED, "inline flag or extension"};
                }
            }
            if (++depth_ > 200) throw ParseError{SG_E_UNSUPPORTED, "nesting too deep"};
            NodeP r = alt(inner_nc);
            --depth_;
            if (peek() != ')') throw ParseError{SG_E_INVAL, "missing )"};
            ++i_;
            atom_grouped_ = true;
            return r;
        }
        if (c == ')') throw ParseError{SG_E_INVAL, "unbalanced parenthesis"};
        if (c == '*' || c == '+' || c == '?') throw ParseError{SG_E_INVAL, "nothing to repeat"};
        if (c == '{') {
            int lo, hi;
            uint32_t len;
            if (quant_brace(&lo, &hi, &len)) throw ParseError{SG_E_INVAL, "nothing to repeat"};
        }
        ++i_;
        if (c == '[') return klass(nc);
        if (c == '.') { ByteSet s; s.set(); s.reset('\n'); return lit(s, false); }
        if (c == '^') return mk(Node::BOL);
        if (c == '$') return mk(Node::EOL);
        if (c == '\\') {
            ByteSet s;
            int b;
            Node::Kind an;
            if (escape(false, &s, &b, &an)) return lit(s, false);
            if (an != Node::EMPTY) return mk(an);
            ByteSet one;
            one.set(b);
            return lit(one, nc);
        }
        ByteSet one;
        one.set(c);
        return lit(one, nc);
    }
};

// ------------------------------------------------------------------ NFA
struct NState {
    enum Type : uint8_t { CHAR, EPS, SPLIT, BOL, EOL, WB, NWB, MATCH } type;
    int out = -1, out2 = -1;
    int set = -1;  // CHAR: index into sets
    int pid = -1;  // MATCH
};

struct NFA {
    std::vector<NState> st;
    std::vector<ByteSet> sets;
    bool has_word_assert = false;
    size_t limit = 400000;
    int add(NState::Type t) {
        if (st.size() >= limit) throw ParseError{SG_E_STATES, "NFA too large"};
        NState s;
        s.type = t;
        st.push_back(s);
        return (int)st.size() - 1;
    }
};

struct Frag {
    int start, end;  // end: an EPS state whose out is patched
};

static Frag build(NFA &A, const Node *n) {
    switch (n->kind) {
        case Node::LIT: {
            int e = A.add(NState::EPS);
            int s = A.add(NState::CHAR);
            A.sets.push_back(n->set);
            A.st[s].set = (int)A.sets.size() - 1;
            A.st[s].out = e;
            return {s, e};
        }
        case Node::EMPTY: {
            int e = A.add(NState::EPS);
            return {e, e};
        }
        case Node::BOL:
        case Node::EOL:
        case Node::WB:
        case Node::NWB: {
            int e = A.add(NState::EPS);
            const NState::Type t = n->kind == Node::BOL ? NState::BOL
                                 : n->kind == Node::EOL ? NState::EOL
                                 : n->kind == Node::WB  ? NState::WB : NState::NWB;
            int s = A.add(t);
            A.st[s].out = e;
            if (t == NState::WB || t == NState::NWB) A.has_word_assert = true;
            return {s, e};
        }
        case Node::CAT: {
            Frag f = build(A, n->kids[0].get());
            for (size_t k = 1; k < n->kids.size(); ++k) {
                Frag g = build(A, n->kids[k].get());
                A.st[f.end].out = g.start;
                f.end = g.end;
            }
            return f;
        }
        case Node::ALT: {
            int e = A.add(NState::EPS);
            int s = -1;
            for (size_t k = 0; k < n->kids.size(); ++k) {
                Frag g = build(A, n->kids[k].get());
                A.st[g.end].out = e;
                if (s < 0) {
                    s = g.start;
                } else {
                    int sp = A.add(NState::SPLIT);
                    A.st[sp].out = s;
                    A.st[sp].out2 = g.start;
                    s = sp;
                }
            }
            return {s, e};
        }
        case Node::REP: {
            const Node *c = n->kids[0].get();
            int e0 = A.add(NState::EPS);
            Frag f{e0, e0};
            for (int k = 0; k < n->lo; ++k) {
                Frag g = build(A, c);
                A.st[f.end].out = g.start;
                f.end = g.end;
            }
            if (n->hi < 0) {
                Frag g = build(A, c);
                int sp = A.add(NState::SPLIT);
                int e = A.add(NState::EPS);
                A.st[sp].out = g.start;
                A.st[sp].out2 = e;
                A.st[g.end].out = sp;
                A.st[f.end].out = sp;
                f.end = e;
            } else {
                int e = A.add(NState::EPS);
                for (int k = n->lo; k < n->hi; ++k) {
                    Frag g = build(A, c);
                    int sp = A.add(NState::SPLIT);
                    A.st[sp].out = g.start;
                    A.st[sp].out2 = e;
                    A.st[f.end].out = sp;
                    f.end = g.end;
                }
                A.st[f.end].out = e;
                f.end = e;
            }
            return f;
        }
    }
    return {-1, -1};
}

// ------------------------------------------------------------------ subset construction
struct VecHash {
    size_t operator()(const std::vector<int> &v) const {
        uint64_t h = 1469598103934665603ull;
        for (int x : v) { h ^= (uint64_t)(uint32_t)x; h *= 1099511628211ull; }
        return (size_t)h;
    }
};

// DFA state = (canonical NFA set, previous byte is a word byte). Canonical sets keep CHAR
// and MATCH states plus the assertion states still waiting for context: EOL (the record
// end) and WB/NWB (the next byte). Consuming byte b first resolves pending word
// assertions with (prev_word, word(b)), then moves on b, then injects the pattern starts
// again (unanchored search). MATCH states reached while resolving count as accepted on
// entering the successor.
class SubsetBuilder {
  public:
    SubsetBuilder(const NFA &A, const std::vector<int> &starts, uint32_t budget, bool anchored = false)
        : A_(A), starts_(starts), budget_(budget), anchored_(anchored), mark_(A.st.size(), 0) {}

    bool run(RegexDFA *out) {
        std::vector<ByteSet> sets = A_.sets;
        ByteSet wordset;
        for (int c = '0'; c <= '9'; ++c) wordset.set(c);
        for (int c = 'a'; c <= 'z'; ++c) { wordset.set(c); wordset.set(c - 32); }
        wordset.set('_');
        if (A_.has_word_assert) sets.push_back(wordset);
        std::vector<std::vector<uint64_t>> sig(256);
        const size_t ns = sets.size();
        for (int b = 0; b < 256; ++b) sig[b].assign((ns + 63) / 64 + 1, 0);
        for (size_t k = 0; k < ns; ++k)
            for (int b = 0; b < 256; ++b)
                if (sets[k][b]) sig[b][k / 64] |= 1ull << (k % 64);
        std::map<std::vector<uint64_t>, int> cid;
        for (int b = 0; b < 256; ++b) {
            auto it = cid.find(sig[b]);
            int c;
            if (it == cid.end()) { c = (int)cid.size(); cid[sig[b]] = c; } else { c = it->second; }
            out->cls[b] = (uint8_t)c;
            if (rep_.size() <= (size_t)c) rep_.push_back(b);
        }
        const uint32_t nbc = (uint32_t)cid.size();
        const uint32_t C = nbc + 1;  // + EOL column
        out->n_classes = C;
        out->eol_class = nbc;
        std::vector<int> init = closure(starts_, true, false, false, false, false);
        start_nb_ = closure(starts_, false, false, false, false, false);
        struct DS { std::vector<int> set; bool pw; bool term; };
        std::vector<DS> states;
        std::vector<std::vector<uint32_t>> acc;
        std::unordered_map<std::vector<int>, uint32_t, VecHash> id;
        auto keyof = [](const std::vector<int> &s, bool pw) {
            std::vector<int> k = s;
            k.push_back(pw ? -2 : -3);
            return k;
        };
        states.push_back({{}, false, false});  // 0: dead
        acc.push_back({});
        auto intern = [&](std::vector<int> &&s, bool pw) -> int64_t {
            if (s.empty()) return 0;
            std::vector<int> k = keyof(s, pw);
            auto it = id.find(k);
            if (it != id.end()) return it->second;
            if (states.size() >= budget_) return -1;
            const uint32_t q = (uint32_t)states.size();
            acc.push_back(accepts(s));
            id.emplace(std::move(k), q);
            states.push_back({std::move(s), pw, false});
            return q;
        };
        if (intern(std::move(init), false) != 1) return false;  // state 1 = start
        out->anchored = anchored_;
        if (anchored_) {  // start states for a search starting after a non-word / word byte
            for (int w = 0; w < 2; ++w) {
                const int64_t t = intern(std::vector<int>(start_nb_), w != 0);
                if (t < 0) return false;
                out->mid_start[w] = (uint32_t)t;
            }
        }
        std::vector<uint32_t> delta;
        std::map<std::vector<uint32_t>, uint32_t> eol_term;
        for (size_t q = 1; q < states.size(); ++q) {
            if (states[q].term) continue;
            const std::vector<int> cur = states[q].set;
            const bool pw = states[q].pw;
            std::vector<uint32_t> row(C, 0);
            for (uint32_t c = 0; c < nbc; ++c) {
                const int b = rep_[c];
                const bool nw = wordset[b];
                std::vector<int> res = cur;
                std::vector<int> newly;
                if (A_.has_word_assert) {
                    res = closure(cur, false, false, true, pw, nw);
                    for (int s : res)
                        if (A_.st[s].type == NState::MATCH && !std::binary_search(cur.begin(), cur.end(), s)) newly.push_back(s);
                }
                std::vector<int> nx = closure(move(res, b), false, false, false, false, false);
                if (!anchored_) nx = merge(nx, start_nb_);
                if (!newly.empty()) nx = merge(nx, newly);
                int64_t t = intern(std::move(nx), nw);
                if (t < 0) return false;
                row[c] = (uint32_t)t;
            }
            // end of record: EOL assertions hold, the next byte counts as non-word
            std::vector<uint32_t> ea;
            {
                std::vector<int> fin = closure(cur, false, true, true, pw, false);
                std::vector<uint32_t> all = accepts(fin), had = acc[q];
                std::set_difference(all.begin(), all.end(), had.begin(), had.end(), std::back_inserter(ea));
            }
            uint32_t t = 0;
            if (!ea.empty()) {
                auto it = eol_term.find(ea);
                if (it == eol_term.end()) {
                    if (states.size() >= budget_) return false;
                    t = (uint32_t)states.size();
                    states.push_back({{}, false, true});
                    acc.push_back(ea);
                    eol_term[ea] = t;
                } else {
                    t = it->second;
                }
            }
            row[nbc] = t;
            delta.resize(states.size() * C, 0);
            std::copy(row.begin(), row.end(), delta.begin() + q * C);
        }
        const uint32_t S = (uint32_t)states.size();
        delta.resize((size_t)S * C, 0);
        out->n_states = S;
        out->delta = std::move(delta);
        out->acc_off.assign(S + 1, 0);
        for (uint32_t q = 0; q < S; ++q) out->acc_off[q + 1] = out->acc_off[q] + (uint32_t)acc[q].size();
        out->acc_ids.clear();
        for (uint32_t q = 0; q < S; ++q) out->acc_ids.insert(out->acc_ids.end(), acc[q].begin(), acc[q].end());
        return true;
    }

  private:
    const NFA &A_;
    std::vector<int> starts_, start_nb_;
    uint32_t budget_;
    bool anchored_;
    std::vector<int> rep_;
    std::vector<uint32_t> mark_;
    uint32_t gen_ = 0;

    static std::vector<int> merge(const std::vector<int> &a, const std::vector<int> &b) {
        std::vector<int> r;
        r.reserve(a.size() + b.size());
        std::set_union(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(r));
        return r;
    }
    // epsilon closure; assertions whose context is unknown stay in the set (pending)
    std::vector<int> closure(const std::vector<int> &seed, bool bol, bool eol, bool wknown, bool pw, bool nw) {
        ++gen_;
        std::vector<int> stack(seed.begin(), seed.end()), out;
        while (!stack.empty()) {
            int s = stack.back();
            stack.pop_back();
            if (s < 0 || mark_[s] == gen_) continue;
            mark_[s] = gen_;
            const NState &n = A_.st[s];
            switch (n.type) {
                case NState::CHAR: out.push_back(s); break;
                case NState::MATCH: out.push_back(s); break;
                case NState::EPS: stack.push_back(n.out); break;
                case NState::SPLIT: stack.push_back(n.out2); stack.push_back(n.out); break;
                case NState::BOL: if (bol) stack.push_back(n.out); break;
                case NState::EOL: if (eol) stack.push_back(n.out); else out.push_back(s); break;
                case NState::WB:
                    if (!wknown) out.push_back(s);
                    else if (pw != nw) stack.push_back(n.out);
                    break;
                case NState::NWB:
                    if (!wknown) out.push_back(s);
                    else if (pw == nw) stack.push_back(n.out);
                    break;
            }
        }
        std::sort(out.begin(), out.end());
        return out;
    }
    std::vector<int> move(const std::vector<int> &S, int byte) {
        std::vector<int> r;
        for (int s : S) {
            const NState &n = A_.st[s];
            if (n.type == NState::CHAR && A_.sets[n.set][byte]) r.push_back(n.out);
        }
        return r;
    }
    std::vector<uint32_t> accepts(const std::vector<int> &S) {
        std::vector<uint32_t> r;
        for (int s : S)
            if (s >= 0 && A_.st[s].type == NState::MATCH) r.push_back((uint32_t)A_.st[s].pid);
        std::sort(r.begin(), r.end());
        r.erase(std::unique(r.begin(), r.end()), r.end());
        return r;
    }
};

struct Pat {
    uint32_t id;
    NodeP ast;
};

static int parse_one(const uint8_t *p, uint32_t len, bool nocase, NodeP *out) {
    try {
        Parser ps(p, len, nocase);
        *out = ps.parse();
        return SG_OK;
    } catch (const ParseError &e) {
        set_error("regex: %s", e.msg);
        return e.code;
    }
}

static int build_group(const std::vector<Pat *> &ps, uint32_t budget, RegexDFA *out, bool *fits,
                       bool anchored = false) {
    try {
        NFA A;
        std::vector<int> starts;
        for (Pat *p : ps) {
            Frag f = build(A, p->ast.get());
            int m = A.add(NState::MATCH);
            A.st[m].pid = (int)p->id;
            A.st[f.end].out = m;
            starts.push_back(f.start);
        }
        SubsetBuilder sb(A, starts, budget, anchored);
        *fits = sb.run(out);
        return SG_OK;
    } catch (const ParseError &e) {
        set_error("regex: %s", e.msg);
        return e.code;
    }
}

// Groups hold at most 64 patterns (the matcher keeps a per-record accept mask in one
// 64-bit register) and at most `budget` states.
static int build_split(std::vector<Pat *> ps, uint32_t budget, std::vector<RegexDFA> *out) {
    RegexDFA d;
    bool fits = false;
    int rc = ps.size() <= 64 ? build_group(ps, budget, &d, &fits) : SG_OK;
    if (rc != SG_OK) return rc;
    if (fits) {
        out->push_back(std::move(d));
        return SG_OK;
    }
    if (ps.size() == 1) {
        if (budget < 65535) return build_split(ps, 65535, out);
        set_error("regex signature %u needs more than %u DFA states", ps[0]->id, budget);
        return SG_E_STATES;
    }
    std::vector<Pat *> a(ps.begin(), ps.begin() + ps.size() / 2), b(ps.begin() + ps.size() / 2, ps.end());
    rc = build_split(a, budget, out);
    if (rc != SG_OK) return rc;
    return build_split(b, budget, out);
}

// Small unfiltered sets are packed first-fit (largest single DFA first) into groups whose
// whole transition table fits the matcher's LDS hot-row budget (states x classes x 2 B
// <= 64 KiB) and the state budget: every group costs one pass over the text, and a table
// that spills rows to L2 costs a dependent L2 load on the cold steps. (The C4 set's 20
// factor-less signatures: 5 halving-split groups, 2 of them over the LDS budget -> packed.)
constexpr uint64_t PACK_TABLE_BYTES = 64 * 1024;
static uint64_t table_bytes(const RegexDFA &d) { return (uint64_t)d.n_states * d.n_classes * 2; }

static int build_pack(std::vector<Pat *> ps, uint32_t budget, std::vector<RegexDFA> *out) {
    if (ps.size() > 128) return build_split(ps, budget, out);
    std::vector<std::pair<uint64_t, Pat *>> order;
    for (Pat *p : ps) {
        RegexDFA d;
        bool fits = false;
        int rc = build_group({p}, budget, &d, &fits);
        if (rc != SG_OK) return rc;
        order.push_back({fits ? table_bytes(d) : ~0ull, p});
    }
    std::stable_sort(order.begin(), order.end(), [](const auto &a, const auto &b) { return a.first > b.first; });
    std::vector<std::vector<Pat *>> groups;
    std::vector<RegexDFA> dfas;
    for (auto &op : order) {
        bool placed = false;
        for (size_t g = 0; g < groups.size() && !placed && op.first <= PACK_TABLE_BYTES; ++g) {
            if (groups[g].size() >= 64 || table_bytes(dfas[g]) > PACK_TABLE_BYTES) continue;
            std::vector<Pat *> trial = groups[g];
            trial.push_back(op.second);
            RegexDFA d;
            bool fits = false;
            int rc = build_group(trial, budget, &d, &fits);
            if (rc != SG_OK) return rc;
            if (fits && table_bytes(d) <= PACK_TABLE_BYTES) {
                groups[g] = std::move(trial);
                dfas[g] = std::move(d);
                placed = true;
            }
        }
        if (!placed) {
            std::vector<RegexDFA> one;
            int rc = build_split({op.second}, budget, &one);
            if (rc != SG_OK) return rc;
            groups.push_back({op.second});
            dfas.push_back(std::move(one[0]));
        }
    }
    for (auto &d : dfas) out->push_back(std::move(d));
    return SG_OK;
}

// ------------------------------------------------------------------ literal factors
// For a node: `exact` = every string the node can match (lower-cased, when small), and
// `fac` = a set such that every match of the node contains one of its strings.
struct Sum {
    bool exact_ok = false;
    std::vector<std::string> exact;
    bool fac_ok = false;
    std::vector<std::string> fac;
    // every factor set of a concatenation's parts (score >= FAC_MIN), so the plan can prefer
    // a set that few other signatures share over the merely longest one
    std::vector<std::vector<std::string>> alts;
};
constexpr size_t FAC_MAXALTS = 24;
constexpr size_t FAC_MAXSET = 64, FAC_MAXLEN = 48;
// Shortest factor string a filtered pattern may have. Round 5 measured 4 on C4 (the 25
// three-byte factors of the C4 set: ':99', 'are', 'asp', ... go, with their 27 patterns, to
// the factor-less DFA groups, tools/factor_stats.cpp): the prefilter's third length class
// disappears (re_prefilter 3.54 -> 3.19 ms) but the DFA groups grow from 4 to 7 and
// dfa_match doubles (1.02 -> 2.17 ms): C4 6.88 -> 7.51 ms, fields 54.1 -> 55.9 ms.
#ifndef SG_FAC_MIN
#define SG_FAC_MIN 3
#endif
constexpr int FAC_MIN = SG_FAC_MIN;

static int fac_score(const std::vector<std::string> &f) {
    if (f.empty()) return 0;
    size_t m = f[0].size();
    for (auto &s : f) m = std::min(m, s.size());
    return (int)m;
}
static bool better(const std::vector<std::string> &a, const std::vector<std::string> &b) {
    const int sa = fac_score(a), sb = fac_score(b);
    if (sa != sb) return sa > sb;
    return a.size() < b.size();
}
static void dedupe(std::vector<std::string> &v) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
}
static std::vector<std::string> effective(const Sum &s) {
    std::vector<std::string> best;
    if (s.fac_ok) best = s.fac;
    if (s.exact_ok) {
        bool has_empty = false;
        for (auto &x : s.exact) has_empty |= x.empty();
        if (!has_empty && (best.empty() || better(s.exact, best))) best = s.exact;
    }
    return best;
}

static Sum summarize(const Node *n) {
    Sum r;
    switch (n->kind) {
        case Node::LIT: {
            std::vector<std::string> cs;
            for (int c = 0; c < 256; ++c) {
                if (!n->set[c]) continue;
                int l = (c >= 'A' && c <= 'Z') ? c + 32 : c;
                std::string s(1, (char)l);
                if (std::find(cs.begin(), cs.end(), s) == cs.end()) cs.push_back(s);
                if (cs.size() > 4) break;
            }
            if (cs.size() <= 4) { r.exact_ok = true; r.exact = cs; }
            return r;
        }
        case Node::BOL: case Node::EOL: case Node::WB: case Node::NWB: case Node::EMPTY:
            r.exact_ok = true;
            r.exact = {std::string()};
            return r;
        case Node::CAT: {
            std::vector<std::string> run{std::string()}, best;
            bool all_exact = true;
            auto consider = [&](const std::vector<std::string> &f) {
                if (!f.empty() && fac_score(f) > 0 && (best.empty() || better(f, best))) best = f;
                if (fac_score(f) >= FAC_MIN && r.alts.size() < FAC_MAXALTS) r.alts.push_back(f);
            };
            for (auto &k : n->kids) {
                Sum cs = summarize(k.get());
                consider(effective(cs));
                if (cs.exact_ok && run.size() * cs.exact.size() <= FAC_MAXSET) {
                    std::vector<std::string> nr;
                    bool too_long = false;
                    for (auto &a : run)
                        for (auto &b : cs.exact) {
                            nr.push_back(a + b);
                            too_long |= nr.back().size() > FAC_MAXLEN;
                        }
                    if (!too_long) { dedupe(nr); run = nr; continue; }
                }
                all_exact = false;
                consider(run);
                run = cs.exact_ok ? cs.exact : std::vector<std::string>{std::string()};
            }
            consider(run);
            if (all_exact) { r.exact_ok = true; r.exact = run; }
            if (!best.empty()) { r.fac_ok = true; r.fac = best; }
            return r;
        }
        case Node::ALT: {
            bool all_exact = true, all_fac = true;
            std::vector<std::string> ex, fa;
            for (auto &k : n->kids) {
                Sum cs = summarize(k.get());
                if (cs.exact_ok) ex.insert(ex.end(), cs.exact.begin(), cs.exact.end()); else all_exact = false;
                std::vector<std::string> e = effective(cs);
                if (e.empty()) all_fac = false; else fa.insert(fa.end(), e.begin(), e.end());
            }
            dedupe(ex);
            dedupe(fa);
            if (all_exact && ex.size() <= FAC_MAXSET) { r.exact_ok = true; r.exact = ex; }
            if (all_fac && fa.size() <= FAC_MAXSET) { r.fac_ok = true; r.fac = fa; }
            return r;
        }
        case Node::REP: {
            Sum cs = summarize(n->kids[0].get());
            if (n->lo >= 1) {
                std::vector<std::string> e = effective(cs);
                if (!e.empty()) { r.fac_ok = true; r.fac = e; }
                if (cs.exact_ok && n->lo == n->hi && n->lo <= 4) {
                    std::vector<std::string> run{std::string()};
                    bool ok = true;
                    for (int k = 0; k < n->lo && ok; ++k) {
                        std::vector<std::string> nr;
                        for (auto &a : run)
                            for (auto &b : cs.exact) nr.push_back(a + b);
                        dedupe(nr);
                        ok = nr.size() <= FAC_MAXSET;
                        run = nr;
                    }
                    if (ok) { r.exact_ok = true; r.exact = run; }
                }
            }
            return r;
        }
    }
    return r;
}

}  // namespace

int regex_build_plan(const uint8_t *pats, const uint32_t *offs, uint32_t n, uint32_t flags, RegexPlan *plan) {
    std::vector<Pat> ps(n);
    for (uint32_t i = 0; i < n; ++i) {
        ps[i].id = i;
        try {
            Parser pr(pats + offs[i], offs[i + 1] - offs[i], flags & SG_NOCASE);
            ps[i].ast = pr.parse();
        } catch (const ParseError &e) {
            set_error("regex signature %u: %s", i, e.msg);
            return e.code;
        }
    }
    plan->single_of_pid.assign(n, 0xffffffffu);
    const bool force_anchored = sw_regex_anchored();  // test switch
    std::map<std::string, std::vector<uint32_t>> fac_map;
    std::vector<Pat *> unfiltered;
    // candidate factor sets per pattern; how many patterns could use each string
    std::vector<std::vector<std::vector<std::string>>> cands(n);
    std::vector<std::vector<std::string>> eff(n);
    std::map<std::string, uint32_t> share;
    for (auto &p : ps) {
        Sum sm = summarize(p.ast.get());
        auto &cs = cands[p.id];
        cs = sm.alts;
        eff[p.id] = effective(sm);
        if (!eff[p.id].empty()) cs.push_back(eff[p.id]);
        for (auto &f : cs) dedupe(f);
        std::sort(cs.begin(), cs.end());
        cs.erase(std::unique(cs.begin(), cs.end()), cs.end());
        std::vector<std::string> mine;
        for (auto &f : cs) mine.insert(mine.end(), f.begin(), f.end());
        dedupe(mine);
        for (auto &x : mine) share[x]++;
    }
    for (auto &p : ps) {
        // the least shared set (max over its strings of the number of patterns that could
        // use them), then the longest; the effective set when nothing scores >= 3
        std::vector<std::string> f = eff[p.id];
        uint64_t best_cost = ~0ull;
        for (auto &c : cands[p.id]) {
            if (fac_score(c) < FAC_MIN) continue;
            uint32_t worst = 0;
            for (auto &x : c) worst = std::max(worst, share[x]);
            const uint64_t cost = ((uint64_t)worst << 32) | (uint32_t)(0x7fffffff - fac_score(c));
            if (cost < best_cost) { best_cost = cost; f = c; }
        }
        const bool had = !f.empty();
        // a factor holding '\n' can never occur inside a record: drop it
        f.erase(std::remove_if(f.begin(), f.end(), [](const std::string &s) { return s.find('\n') != std::string::npos; }),
                f.end());
        bool filtered = fac_score(f) >= FAC_MIN || (had && f.empty());
        if (filtered) {
            RegexDFA d;
            bool fits = false;
            std::vector<Pat *> one{&p};
            int rc = force_anchored ? SG_OK : build_group(one, 65535, &d, &fits);
            if (rc != SG_OK) return rc;
            if (!fits) {  // verification runs per candidate: an anchored DFA will do
                d = RegexDFA();
                rc = build_group(one, 65535, &d, &fits, true);
                if (rc != SG_OK) return rc;
            }
            if (!fits) {
                filtered = false;
            } else {
                plan->single_of_pid[p.id] = (uint32_t)plan->singles.size();
                plan->singles.push_back(std::move(d));
                plan->single_pid.push_back(p.id);
                for (auto &s : f) fac_map[s].push_back(p.id);
            }
        }
        if (!filtered) unfiltered.push_back(&p);
    }
    plan->fac_off.assign(1, 0);
    for (auto &kv : fac_map) {
        plan->factors.emplace_back(kv.first.begin(), kv.first.end());
        std::vector<uint32_t> ids = kv.second;
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
        plan->fac_pids.insert(plan->fac_pids.end(), ids.begin(), ids.end());
        plan->fac_off.push_back((uint32_t)plan->fac_pids.size());
    }
    if (!unfiltered.empty()) {
        return build_pack(unfiltered, 4096, &plan->groups);
    }
    return SG_OK;
}

int regex_check(const uint8_t *pat, uint32_t len, uint32_t flags) {
    NodeP n;
    return parse_one(pat, len, flags & SG_NOCASE, &n);
}

int regex_build_set(const uint8_t *pats, const uint32_t *offs, uint32_t n, uint32_t flags,
                    std::vector<RegexDFA> *out) {
    std::vector<Pat> ps(n);
    for (uint32_t i = 0; i < n; ++i) {
        ps[i].id = i;
        int rc = parse_one(pats + offs[i], offs[i + 1] - offs[i], flags & SG_NOCASE, &ps[i].ast);
        if (rc != SG_OK) {
            set_error("regex signature %u: %s", i, "unsupported or invalid (see previous)");
            NodeP tmp;
            parse_one(pats + offs[i], offs[i + 1] - offs[i], flags & SG_NOCASE, &tmp);  // restore message
            return rc;
        }
    }
    std::vector<Pat *> all;
    for (auto &p : ps) all.push_back(&p);
    const uint32_t budget = 4096;
    if (all.empty()) return SG_OK;
    return build_split(all, budget, out);
}

}  // namespace sg
