// bt_regex_dfa.cpp — PAYLOAD filter regex -> byte DFA for the GPU.
//
// The reference evaluates a PAYLOAD filter as
//     std::regex_search(std::string(payload, min(len - off, 100)), std::regex(expr))
// (src/PacketFilter.cpp:288-321) with libstdc++'s ECMAScript grammar. This file
// compiles the regular subset of that grammar into a DFA over bytes that answers the
// same question — "does any substring match?" — in one pass:
//
//   * unanchored search: the NFA start is re-injected at every position, so a DFA
//     state is the set of partial matches alive at that position;
//   * `^` is an assertion true only at position 0, `$` only at the end (no multiline,
//     as regex_search with default flags); each DFA state records whether a match is
//     complete now (search succeeds: stop), complete if the input ends here, or
//     impossible from here on (stop);
//   * character sets follow libstdc++ exactly as measured (`.` = all but \n \r; \s
//     = 09-0d, 20; \w / \d ASCII; ranges compared as signed char).
//
// Anything outside the modelled subset — backreferences, lookaheads, \b \B, \c \u,
// POSIX [[:classes:]], escapes of letters libstdc++ treats idiosyncratically, more
// than 255 DFA states — returns BT_E_NOT_IMPLEMENTED and the filter stays on the
// host (std::regex), as before. Only patterns std::regex itself accepts reach here
// (the filter compiler probes first), so the parser never needs error recovery for
// patterns the reference rejects. Agreement with std::regex is fuzzed in
// tests/cpp/test_regex_dfa.cpp.
//
// Blob layout (4-B aligned, little endian), shared by the host executor below and
// the kernel (bt_kernels.hip, eval_payload). States 0..K-1 are live; K is the ACCEPT
// sink (a match completed: search succeeds) and K+1 the DEAD sink (no match can
// complete any more), so the per-byte loop exits on `q >= K` without a table read.
//   u16 K, u16 C          C = 256: `next` is indexed by the byte itself (one dependent
//                         LDS read per byte); otherwise C byte classes via cls[]
//   u8  init, u8 empty    init state (may be a sink); empty = match on the empty input
//   u8  pairs, u8 P       pairs = 1: a two-byte table follows (P byte classes)
//   u8  endacc[K] (pad 4) 1 = a match completes if the input ends in this state
//   u8  cls[256]          only when C != 256
//   u8  next[K * C]       (pad 4)
//   u8  clsp[256]         pairs only: byte -> class of the two-byte table
//   u8  pair[K * P * P]   pairs only: the state after two bytes (a sink after the first
//                         stays), so the walk's dependent chain is half as long
#include <algorithm>
#include <bitset>
#include <cstring>
#include <map>
#include <regex>
#include <string>
#include <vector>

#include "beatrice_gpu_bench.h"

namespace {

using Set = std::bitset<256>;

constexpr int kMaxNfa = 6000;
constexpr int kMaxDfa = 255;
constexpr int kMaxRepeat = 100;   // payload windows are <= 100 bytes

// ------------------------------------------------------------------ parse -> AST

struct Node {
    enum T { SET, CAT, ALT, REP, BOL, EOL, EMPTY } t;
    Set set;
    std::vector<int> kids;
    int lo = 0, hi = 0;   // REP: hi < 0 = unbounded
};

struct Unsupported {};

class Parser {
public:
    explicit Parser(const std::string& p) : p_(p) {}
    std::vector<Node> nodes;

    int parse() {
        const int r = disjunction();
        if (i_ != p_.size()) throw Unsupported{};
        return r;
    }

private:
    const std::string& p_;
    size_t i_ = 0;

    bool more() const { return i_ < p_.size(); }
    unsigned char peek() const { return (unsigned char)p_[i_]; }

    int add(Node n) {
        nodes.push_back(std::move(n));
        return (int)nodes.size() - 1;
    }
    int set_node(const Set& s) {
        Node n{Node::SET};
        n.set = s;
        return add(n);
    }

    int disjunction() {
        std::vector<int> alts{alternative()};
        while (more() && peek() == '|') {
            ++i_;
            alts.push_back(alternative());
        }
        if (alts.size() == 1) return alts[0];
        Node n{Node::ALT};
        n.kids = alts;
        return add(n);
    }

    int alternative() {
        std::vector<int> terms;
        while (more() && peek() != '|' && peek() != ')') terms.push_back(term());
        if (terms.empty()) return add(Node{Node::EMPTY});
        if (terms.size() == 1) return terms[0];
        Node n{Node::CAT};
        n.kids = terms;
        return add(n);
    }

    int term() {
        const unsigned char c = peek();
        if (c == '^' || c == '$') {
            ++i_;
            if (more() && (peek() == '*' || peek() == '+' || peek() == '?' || peek() == '{'))
                throw Unsupported{};   // quantified assertion
            return add(Node{c == '^' ? Node::BOL : Node::EOL});
        }
        int a = atom();
        while (more()) {   // libstdc++ accepts stacked quantifiers (a**): apply each in turn
            int lo, hi;
            if (!quantifier(lo, hi)) break;
            Node n{Node::REP};
            n.kids = {a};
            n.lo = lo;
            n.hi = hi;
            a = add(n);
        }
        return a;
    }

    bool number(int& v) {
        if (!more() || !isdigit(peek())) return false;
        long x = 0;
        while (more() && isdigit(peek())) {
            x = x * 10 + (peek() - '0');
            if (x > 100000) throw Unsupported{};
            ++i_;
        }
        v = (int)x;
        return true;
    }

    bool quantifier(int& lo, int& hi) {
        const unsigned char c = peek();
        if (c == '*') { lo = 0; hi = -1; ++i_; }
        else if (c == '+') { lo = 1; hi = -1; ++i_; }
        else if (c == '?') { lo = 0; hi = 1; ++i_; }
        else if (c == '{') {
            ++i_;
            if (!number(lo)) throw Unsupported{};
            hi = lo;
            if (more() && peek() == ',') {
                ++i_;
                if (!number(hi)) hi = -1;
            }
            if (!more() || peek() != '}') throw Unsupported{};
            ++i_;
            if (lo > kMaxRepeat || hi > kMaxRepeat) throw Unsupported{};
        } else {
            return false;
        }
        if (more() && peek() == '?') ++i_;   // lazy: the same language
        return true;
    }

    static Set range(int a, int b) {
        Set s;
        for (int x = a; x <= b; ++x) s.set(x & 0xFF);
        return s;
    }
    static Set digit() { return range('0', '9'); }
    static Set word() { return range('0', '9') | range('A', 'Z') | range('a', 'z') | range('_', '_'); }
    static Set space() { return range(9, 13) | range(' ', ' '); }

    static int hexval(unsigned char c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }

    // After a backslash. Returns true with `single` set for a one-byte escape, or false
    // with `cls` set for a class escape (\d \w \s and negations).
    bool escape(bool in_class, int& single, Set& cls) {
        if (!more()) throw Unsupported{};
        const unsigned char c = peek();
        ++i_;
        switch (c) {
        case 'd': cls = digit(); return false;
        case 'D': cls = ~digit(); return false;
        case 'w': cls = word(); return false;
        case 'W': cls = ~word(); return false;
        case 's': cls = space(); return false;
        case 'S': cls = ~space(); return false;
        case 't': single = 9; return true;
        case 'n': single = 10; return true;
        case 'v': single = 11; return true;
        case 'f': single = 12; return true;
        case 'r': single = 13; return true;
        case 'b':
            if (!in_class) throw Unsupported{};   // word boundary
            single = 8;
            return true;
        case '0':
            if (more() && isdigit(peek())) throw Unsupported{};
            single = 0;
            return true;
        case 'x': {
            if (i_ + 2 > p_.size()) throw Unsupported{};
            const int h = hexval((unsigned char)p_[i_]), l = hexval((unsigned char)p_[i_ + 1]);
            if (h < 0 || l < 0) throw Unsupported{};
            i_ += 2;
            single = h * 16 + l;
            return true;
        }
        default:
            if (isalnum(c) || c == '_') throw Unsupported{};   // \1.. \c \u \B and letters
            single = c;                                         // identity escape
            return true;
        }
    }

    Set char_class() {   // after '['
        bool neg = false;
        if (more() && peek() == '^') {
            neg = true;
            ++i_;
        }
        Set s;
        bool first = true;
        while (true) {
            if (!more()) throw Unsupported{};
            unsigned char c = peek();
            if (c == ']') {
                ++i_;
                break;
            }
            if (c == '[') throw Unsupported{};   // [[:alpha:]] and friends
            int lo = -1;
            Set cls;
            ++i_;
            if (c == '\\') {
                int single = 0;
                if (escape(true, single, cls)) lo = single;
            } else {
                lo = c;
            }
            (void)first;
            first = false;
            if (lo < 0) {   // class escape: a following '-' is literal or an error
                if (more() && peek() == '-' && i_ + 1 < p_.size() && p_[i_ + 1] != ']') throw Unsupported{};
                s |= cls;
                continue;
            }
            if (more() && peek() == '-' && i_ + 1 < p_.size() && p_[i_ + 1] != ']') {
                ++i_;
                unsigned char d = peek();
                ++i_;
                int hi;
                if (d == '\\') {
                    int single = 0;
                    Set c2;
                    if (!escape(true, single, c2)) throw Unsupported{};
                    hi = single;
                } else if (d == '[') {
                    throw Unsupported{};
                } else {
                    hi = d;
                }
                // libstdc++ compares range ends as (signed) char
                const int slo = (int)(signed char)lo, shi = (int)(signed char)hi;
                if (slo > shi) throw Unsupported{};   // std::regex rejects these itself
                for (int v = slo; v <= shi; ++v) s.set((unsigned char)(signed char)v);
            } else {
                s.set(lo);
            }
        }
        return neg ? ~s : s;
    }

    int atom() {
        const unsigned char c = peek();
        switch (c) {
        case '(': {
            ++i_;
            if (more() && peek() == '?') {
                if (i_ + 1 < p_.size() && p_[i_ + 1] == ':') i_ += 2;
                else throw Unsupported{};   // lookahead
            }
            const int r = disjunction();
            if (!more() || peek() != ')') throw Unsupported{};
            ++i_;
            return r;
        }
        case '.': {
            ++i_;
            Set s;
            s.set();
            s.reset('\n');
            s.reset('\r');
            return set_node(s);
        }
        case '[':
            ++i_;
            return set_node(char_class());
        case '\\': {
            ++i_;
            int single = 0;
            Set cls;
            if (escape(false, single, cls)) {
                Set s;
                s.set(single);
                return set_node(s);
            }
            return set_node(cls);
        }
        case '*': case '+': case '?': case '{': case ')': case '|':
            throw Unsupported{};
        default: {
            ++i_;
            Set s;
            s.set(c);
            return set_node(s);
        }
        }
    }
};

// ------------------------------------------------------------------ AST -> NFA

struct NState {
    enum T : uint8_t { SET, EPS, SPLIT, BOL, EOL, MATCH } t;
    int set_id = -1;
    int out = -1, out1 = -1;
};

class Nfa {
public:
    std::vector<NState> st;
    std::vector<Set> sets;

    int make(NState::T t) {
        if ((int)st.size() >= kMaxNfa) throw Unsupported{};
        st.push_back(NState{t});
        return (int)st.size() - 1;
    }

    // fragment: entry state, exit EPS state (out unpatched)
    std::pair<int, int> build(const std::vector<Node>& ast, int id) {
        const Node& n = ast[id];
        switch (n.t) {
        case Node::SET: {
            const int s = make(NState::SET), e = make(NState::EPS);
            st[s].set_id = (int)sets.size();
            sets.push_back(n.set);
            st[s].out = e;
            return {s, e};
        }
        case Node::EMPTY: {
            const int e = make(NState::EPS);
            return {e, e};
        }
        case Node::BOL:
        case Node::EOL: {
            const int s = make(n.t == Node::BOL ? NState::BOL : NState::EOL), e = make(NState::EPS);
            st[s].out = e;
            return {s, e};
        }
        case Node::CAT: {
            auto f = build(ast, n.kids[0]);
            for (size_t k = 1; k < n.kids.size(); ++k) {
                auto g = build(ast, n.kids[k]);
                st[f.second].out = g.first;
                f.second = g.second;
            }
            return f;
        }
        case Node::ALT: {
            const int e = make(NState::EPS);
            int entry = -1, prev_split = -1;
            for (size_t k = 0; k < n.kids.size(); ++k) {
                auto g = build(ast, n.kids[k]);
                st[g.second].out = e;
                if (k + 1 < n.kids.size()) {
                    const int sp = make(NState::SPLIT);
                    st[sp].out = g.first;
                    if (prev_split >= 0) st[prev_split].out1 = sp;
                    else entry = sp;
                    prev_split = sp;
                } else {
                    if (prev_split >= 0) st[prev_split].out1 = g.first;
                    else entry = g.first;
                }
            }
            return {entry, e};
        }
        case Node::REP: {
            const int e0 = make(NState::EPS);
            int entry = e0, tail = e0;
            for (int k = 0; k < n.lo; ++k) {
                auto g = build(ast, n.kids[0]);
                st[tail].out = g.first;
                tail = g.second;
            }
            if (n.hi < 0) {   // x*
                auto g = build(ast, n.kids[0]);
                const int sp = make(NState::SPLIT), e = make(NState::EPS);
                st[tail].out = sp;
                st[sp].out = g.first;
                st[sp].out1 = e;
                st[g.second].out = sp;
                return {entry, e};
            }
            const int e = make(NState::EPS);
            for (int k = n.lo; k < n.hi; ++k) {   // nested optionals
                auto g = build(ast, n.kids[0]);
                const int sp = make(NState::SPLIT);
                st[tail].out = sp;
                st[sp].out = g.first;
                st[sp].out1 = e;
                tail = g.second;
            }
            st[tail].out = e;
            return {entry, e};
        }
        }
        throw Unsupported{};
    }

    // epsilon closure; BOL edges only when bol, EOL edges only when eol
    void closure(std::vector<int>& set, bool bol, bool eol) const {
        std::vector<char> seen(st.size(), 0);
        std::vector<int> stack(set.begin(), set.end());
        set.clear();
        while (!stack.empty()) {
            const int s = stack.back();
            stack.pop_back();
            if (s < 0 || seen[s]) continue;
            seen[s] = 1;
            set.push_back(s);
            const NState& n = st[s];
            switch (n.t) {
            case NState::EPS: stack.push_back(n.out); break;
            case NState::SPLIT: stack.push_back(n.out); stack.push_back(n.out1); break;
            case NState::BOL: if (bol) stack.push_back(n.out); break;
            case NState::EOL: if (eol) stack.push_back(n.out); break;
            default: break;
            }
        }
        std::sort(set.begin(), set.end());
    }

    bool has_match(const std::vector<int>& set) const {
        for (int s : set)
            if (st[s].t == NState::MATCH) return true;
        return false;
    }
};

struct Dfa {
    int n_classes = 0, init = 0;
    uint8_t cls[256];
    std::vector<uint8_t> acc;
    std::vector<uint8_t> next;   // [state][class]
};

Dfa build_dfa(const std::string& pattern) {
    Parser ps(pattern);
    const int root = ps.parse();
    Nfa nfa;
    auto frag = nfa.build(ps.nodes, root);
    const int match = nfa.make(NState::MATCH);
    nfa.st[frag.second].out = match;
    const int start = frag.first;

    // byte classes: bytes with the same membership in every set are interchangeable
    Dfa d;
    {
        std::map<std::vector<bool>, int> sig;
        for (int b = 0; b < 256; ++b) {
            std::vector<bool> v(nfa.sets.size());
            for (size_t k = 0; k < nfa.sets.size(); ++k) v[k] = nfa.sets[k].test(b);
            auto it = sig.find(v);
            if (it == sig.end()) it = sig.emplace(v, (int)sig.size()).first;
            d.cls[b] = (uint8_t)it->second;
        }
        d.n_classes = (int)sig.size();
    }
    std::vector<int> rep(d.n_classes, -1);   // a representative byte per class
    for (int b = 0; b < 256; ++b)
        if (rep[d.cls[b]] < 0) rep[d.cls[b]] = b;

    std::vector<int> inject{start};
    nfa.closure(inject, false, false);
    std::vector<int> init{start};
    nfa.closure(init, true, false);

    std::map<std::vector<int>, int> ids;
    std::vector<std::vector<int>> sets;
    auto intern = [&](const std::vector<int>& s) {
        auto it = ids.find(s);
        if (it != ids.end()) return it->second;
        if ((int)sets.size() >= kMaxDfa) throw Unsupported{};
        ids.emplace(s, (int)sets.size());
        sets.push_back(s);
        return (int)sets.size() - 1;
    };
    d.init = intern(init);
    for (size_t q = 0; q < sets.size(); ++q) {
        for (int c = 0; c < d.n_classes; ++c) {
            std::vector<int> mv;
            for (int s : sets[q]) {
                const NState& n = nfa.st[s];
                if (n.t == NState::SET && nfa.sets[n.set_id].test(rep[c])) mv.push_back(n.out);
            }
            nfa.closure(mv, false, false);
            std::vector<int> u;
            std::set_union(mv.begin(), mv.end(), inject.begin(), inject.end(), std::back_inserter(u));
            const int to = intern(u);
            if (d.next.size() < (q + 1) * (size_t)d.n_classes) d.next.resize((q + 1) * (size_t)d.n_classes);
            d.next[q * d.n_classes + c] = (uint8_t)to;
        }
    }
    const int S = (int)sets.size();
    d.next.resize((size_t)S * d.n_classes);
    d.acc.assign(S, 0);
    for (int q = 0; q < S; ++q) {
        if (nfa.has_match(sets[q])) d.acc[q] |= 1;
        std::vector<int> e = sets[q];
        nfa.closure(e, false, true);
        if (nfa.has_match(e)) d.acc[q] |= 2;
    }
    {
        std::vector<int> e = init;
        nfa.closure(e, true, true);
        if (nfa.has_match(e)) d.acc[d.init] |= 8;
    }
    // states from which no match can complete: stop early with false
    std::vector<char> live(S, 0);
    for (int q = 0; q < S; ++q) live[q] = (d.acc[q] & 3) != 0;
    for (bool changed = true; changed;) {
        changed = false;
        for (int q = 0; q < S; ++q) {
            if (live[q]) continue;
            for (int c = 0; c < d.n_classes && !live[q]; ++c)
                if (live[d.next[q * d.n_classes + c]]) live[q] = changed = true;
        }
    }
    for (int q = 0; q < S; ++q)
        if (!live[q]) d.acc[q] |= 4;
    return d;
}

// Live states, sinks and table shape of the serialized DFA.
struct Packed {
    int K = 0, C = 0, init = 0, empty = 0, P = 0;
    std::vector<uint8_t> endacc, cls, next, clsp, pair;
};

constexpr int kPairTableMax = 4096;       // K * P * P bytes: the two-byte table is optional

constexpr int kByteTableMaxStates = 32;   // K * 256 <= 8 KiB: index by the byte, skip cls[]

Packed pack(const Dfa& d, bool pairs) {
    const int S = (int)d.acc.size();
    // live = neither "match complete" (absorbing true) nor "no match possible"
    std::vector<int> id(S, -1);
    int K = 0;
    for (int q = 0; q < S; ++q)
        if (!(d.acc[q] & 1) && !(d.acc[q] & 4)) id[q] = K++;
    if (K + 2 > 256) throw Unsupported{};
    auto map = [&](int q) { return (d.acc[q] & 1) ? K : (d.acc[q] & 4) ? K + 1 : id[q]; };
    Packed p;
    p.K = K;
    p.init = map(d.init);
    p.empty = (d.acc[d.init] >> 3) & 1;
    p.endacc.assign(K, 0);
    for (int q = 0; q < S; ++q)
        if (id[q] >= 0) p.endacc[id[q]] = (d.acc[q] >> 1) & 1;
    const bool bytes = K <= kByteTableMaxStates;
    p.C = bytes ? 256 : d.n_classes;
    if (!bytes) p.cls.assign(d.cls, d.cls + 256);
    p.next.assign((size_t)K * p.C, 0);
    for (int q = 0; q < S; ++q) {
        if (id[q] < 0) continue;
        for (int c = 0; c < p.C; ++c) {
            const int cl = bytes ? d.cls[c] : c;
            p.next[(size_t)id[q] * p.C + c] = (uint8_t)map(d.next[(size_t)q * d.n_classes + cl]);
        }
    }
    const int P = d.n_classes;
    if (pairs && K > 0 && (size_t)K * P * P <= (size_t)kPairTableMax) {
        p.P = P;
        p.clsp.assign(d.cls, d.cls + 256);
        p.pair.assign((size_t)K * P * P, 0);
        for (int q = 0; q < S; ++q) {
            if (id[q] < 0) continue;
            for (int c0 = 0; c0 < P; ++c0) {
                const int t = d.next[(size_t)q * P + c0];
                for (int c1 = 0; c1 < P; ++c1) {
                    const int to = map(t) >= K ? map(t) : map(d.next[(size_t)t * P + c1]);
                    p.pair[((size_t)id[q] * P + c0) * P + c1] = (uint8_t)to;
                }
            }
        }
    }
    return p;
}

uint32_t blob_size(const Packed& p) {
    uint32_t n = 8 + ((p.K + 3) & ~3) + (p.C == 256 ? 0 : 256) + (uint32_t)p.K * p.C;
    if (p.P) n = ((n + 3) & ~3u) + 256 + (uint32_t)p.K * p.P * p.P;
    return n;
}

// ------------------------------------------------------------------ AST -> bit-parallel form
//
// Most payload patterns are a union of linear sequences: byte classes one after another,
// each maybe optional (?) and/or repeatable (+ *), the union maybe anchored at either end —
// "GET|POST", "(?:GET|HEAD) /[^ ]* HTTP" (two sequences once the group is distributed),
// "Host: [a-z0-9.-]+\.com", "^.{0,5}$". Such a union is searched with an extended
// Shift-And over <= 64 positions, one bit per class occurrence (Navarro & Raffinot,
// "Flexible Pattern Matching in Strings", ch. 4): per byte c
//     D = (((D << 1) & NF) | inject | (D & S)) & B[c]      then  D |= (D << 1) & A, R times
// where B[c] marks the positions whose class holds c, S the repeatable ones, A the optional
// ones (the closure skips runs of up to R of them), inject the start of every sequence (at
// every byte; at byte 0 only for ^-anchored ones) and NF clears the first bit of anchored
// sequences so the previous sequence's last bit cannot leak into it. A match ends where a
// sequence's last bit is set (a $-anchored one only after the last byte). The masks B[c]
// depend on the byte alone, so the kernel fetches them ahead and the state chain is a few
// ALU operations per byte instead of a dependent table read.
//
// Blob (16-B aligned like every pool blob; little endian):
//   u16 0xFFFF (no DFA has that many states), u16 W (8 / 16 / 32 / 64: the positions rounded
//   up; the width of a table entry, so small patterns read 1- or 2-byte entries, whose
//   256-entry table spans fewer LDS banks' worth of distinct dwords)
//   u8 m (the longest match in bytes when no class is optional or repeated, else 0),
//   u8 empty (match on the empty input), u8 form (1 search, 2 always true, 3 never),
//   u8 R (closure steps)
//   u32 flags: 1 S != 0, 2 some sequence ^-anchored, 4 every sequence ^-anchored, 8 Fe != 0
//   u8 1 + a byte no class holds (0: none, or it is 0xFF), u8 0 x3
//   u64 Iall, I0, S, A, NF, F, Fe      (I0 = the extra starts at byte 0)
//   u64 pad
//   B[256]: W-bit entries at byte 80
constexpr uint16_t kBitparMagic = 0xFFFF;
constexpr uint32_t kBitparHeader = 80;
constexpr int kBitparMaxSeqs = 64;
constexpr int kBitparMaxR = 8;

struct Item {
    enum K : uint8_t { SET, BOL, EOL } k = SET;
    int set = -1;   // index into Bitpar::sets
    bool opt = false, rep = false;
};
using Seqs = std::vector<std::vector<Item>>;

struct Bitpar {
    const std::vector<Node>& ast;
    std::vector<Set> sets;
    explicit Bitpar(const std::vector<Node>& a) : ast(a) {}

    static Seqs product(const Seqs& a, const Seqs& b) {
        if (a.size() * b.size() > (size_t)kBitparMaxSeqs) throw Unsupported{};
        Seqs r;
        for (const auto& x : a)
            for (const auto& y : b) {
                r.push_back(x);
                r.back().insert(r.back().end(), y.begin(), y.end());
                if (r.back().size() > 64) throw Unsupported{};
            }
        return r;
    }

    Seqs expand(int id) {
        const Node& n = ast[id];
        switch (n.t) {
        case Node::SET: {
            Item it;
            it.set = (int)sets.size();
            sets.push_back(n.set);
            return {{it}};
        }
        case Node::EMPTY: return {{}};
        case Node::BOL: case Node::EOL: {
            Item it;
            it.k = n.t == Node::BOL ? Item::BOL : Item::EOL;
            return {{it}};
        }
        case Node::CAT: {
            Seqs r{{}};
            for (int k : n.kids) r = product(r, expand(k));
            return r;
        }
        case Node::ALT: {
            Seqs r;
            for (int k : n.kids) {
                Seqs e = expand(k);
                r.insert(r.end(), e.begin(), e.end());
                if (r.size() > (size_t)kBitparMaxSeqs) throw Unsupported{};
            }
            return r;
        }
        case Node::REP: {
            const Seqs k = expand(n.kids[0]);
            for (const auto& s : k)
                for (const Item& it : s)
                    if (it.k != Item::SET) throw Unsupported{};   // a repeated assertion
            if (k.size() == 1 && k[0].size() == 1) {   // one class occurrence: copies of it
                const Item x = k[0][0];
                std::vector<Item> s;
                if (n.hi < 0) {
                    for (int c = 0; c + 1 < std::max(n.lo, 1); ++c) s.push_back(x);
                    Item last = x;
                    last.rep = true;
                    if (n.lo == 0) last.opt = true;
                    s.push_back(last);
                } else {
                    for (int c = 0; c < n.hi; ++c) {
                        Item y = x;
                        if (c >= n.lo) y.opt = true;
                        s.push_back(y);
                    }
                }
                if (s.size() > 64) throw Unsupported{};
                return {s};
            }
            if (n.hi < 0) throw Unsupported{};   // (ab)* and the like: the DFA's
            Seqs r;
            for (int cnt = n.lo; cnt <= n.hi; ++cnt) {
                Seqs c{{}};
                for (int j = 0; j < cnt; ++j) c = product(c, k);
                r.insert(r.end(), c.begin(), c.end());
                if (r.size() > (size_t)kBitparMaxSeqs) throw Unsupported{};
            }
            return r;
        }
        }
        throw Unsupported{};
    }
};

struct BitparBlob {
    int W = 32, form = 1, R = 0, empty = 0, longest = 0;
    uint32_t flags = 0;
    uint64_t Iall = 0, I0 = 0, S = 0, A = 0, NF = ~0ull, F = 0, Fe = 0;
    uint64_t B[256] = {};
};

BitparBlob build_bitpar(const std::string& pattern) {
    Parser ps(pattern);
    const int root = ps.parse();
    Bitpar bp(ps.nodes);
    const Seqs all = bp.expand(root);
    struct Lin {
        std::vector<Item> e;   // classes only
        bool bol = false, eol = false;
    };
    std::vector<Lin> keep;
    BitparBlob o;
    for (const auto& s : all) {
        // where the assertions stand: ^ must come before every class, $ after every one
        Lin l;
        bool impossible = false;
        for (int i = 0; i < (int)s.size(); ++i) {
            if (s[i].k == Item::SET) continue;
            bool mand_before = false, mand_after = false, any_before = false, any_after = false;
            for (int j = 0; j < i; ++j)
                if (s[j].k == Item::SET) { any_before = true; mand_before |= !s[j].opt; }
            for (int j = i + 1; j < (int)s.size(); ++j)
                if (s[j].k == Item::SET) { any_after = true; mand_after |= !s[j].opt; }
            if (s[i].k == Item::BOL) {
                if (mand_before) impossible = true;     // ^ after a consumed byte never holds
                else if (any_before) throw Unsupported{};
                else l.bol = true;
            } else {
                if (mand_after) impossible = true;      // $ before a byte to consume
                else if (any_after) throw Unsupported{};
                else l.eol = true;
            }
        }
        if (impossible) continue;
        for (const Item& it : s)
            if (it.k == Item::SET) l.e.push_back(it);
        bool nullable = true;
        for (const Item& it : l.e) nullable &= it.opt;
        if (nullable) {
            o.empty = 1;
            if (!(l.bol && l.eol)) {   // matches the empty string somewhere in any input
                o.form = 2;
                return o;
            }
            if (l.e.empty()) continue;   // ^$: only the empty input
        }
        keep.push_back(std::move(l));
    }
    if (keep.empty()) {
        o.form = 3;
        return o;
    }
    int bit = 0;
    for (const Lin& l : keep) {
        const int m = (int)l.e.size();
        if (bit + m > 64) throw Unsupported{};
        // starts: the first class and every class reachable by skipping optional ones
        uint64_t starts = 0;
        for (int j = 0; j < m; ++j) {
            starts |= 1ull << (bit + j);
            if (!l.e[j].opt) break;
        }
        (l.bol ? o.I0 : o.Iall) |= starts;
        if (l.bol) o.NF &= ~(1ull << bit);
        int run = 0;
        for (int j = 0; j < m; ++j) {
            const Item& it = l.e[j];
            const uint64_t b = 1ull << (bit + j);
            if (it.rep) o.S |= b;
            if (it.opt && j > 0) o.A |= b;   // a sequence's first class is skipped by `starts`
            run = it.opt && j > 0 ? run + 1 : 0;
            o.R = std::max(o.R, run);
            for (int c = 0; c < 256; ++c)
                if (bp.sets[it.set].test(c)) o.B[c] |= b;
        }
        (l.eol ? o.Fe : o.F) |= 1ull << (bit + m - 1);
        o.longest = std::max(o.longest, m);
        bit += m;
    }
    if (o.R > kBitparMaxR) throw Unsupported{};
    o.A &= o.NF;
    o.W = bit <= 8 ? 8 : bit <= 16 ? 16 : bit <= 32 ? 32 : 64;
    o.flags = (o.S ? 1u : 0u) | (o.I0 ? 2u : 0u) | (!o.Iall ? 4u : 0u) | (o.Fe ? 8u : 0u);
    return o;
}

uint32_t bitpar_size(const BitparBlob& o) {
    return o.form != 1 ? kBitparHeader : kBitparHeader + 256u * (uint32_t)(o.W / 8);
}

void bitpar_write(const BitparBlob& o, uint8_t* p) {
    std::memset(p, 0, bitpar_size(o));
    const uint16_t magic = kBitparMagic, w = (uint16_t)o.W;
    std::memcpy(p, &magic, 2);
    std::memcpy(p + 2, &w, 2);
    // the longest match in bytes when every class occurs exactly once (no ?, *, +): the
    // kernel may then search pieces of the window independently (bitpar_chains)
    p[4] = (o.S || o.A || o.longest > 255) ? 0 : (uint8_t)o.longest;
    // 1 + the smallest byte no position's class holds (B[z] == 0), 0 if every byte is in some
    // class: the kernel pads the window with it (bitpar_fast)
    for (int c = 0; c < 256 && o.form == 1; ++c)
        if (!o.B[c]) {
            p[12] = (uint8_t)(c + 1 <= 255 ? c + 1 : 0);
            break;
        }
    p[5] = (uint8_t)o.empty;
    p[6] = (uint8_t)o.form;
    p[7] = (uint8_t)o.R;
    std::memcpy(p + 8, &o.flags, 4);
    const uint64_t m[7] = {o.Iall, o.I0, o.S, o.A, o.NF, o.F, o.Fe};
    std::memcpy(p + 16, m, sizeof(m));
    if (o.form != 1) return;
    const int e = o.W / 8;   // table entry bytes: the state width rounded up to 8/16/32/64 bits
    for (int c = 0; c < 256; ++c) std::memcpy(p + kBitparHeader + e * c, &o.B[c], e);   // little endian
}

// The host executor of a bit-parallel blob: the kernel's loop, byte by byte.
int bitpar_search(const uint8_t* p, const uint8_t* s, uint32_t n) {
    if (n == 0) return p[5];
    if (p[6] != 1) return p[6] == 2;
    uint16_t W;
    std::memcpy(&W, p + 2, 2);
    uint64_t m[7];
    std::memcpy(m, p + 16, sizeof(m));
    const uint64_t Iall = m[0], I0 = m[1], S = m[2], A = m[3], NF = m[4], F = m[5], Fe = m[6];
    const uint32_t R = p[7];
    uint64_t D = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint64_t b = 0;
        std::memcpy(&b, p + kBitparHeader + (W / 8) * s[i], W / 8);
        D = (((D << 1) & NF) | Iall | (i == 0 ? I0 : 0) | (D & S)) & b;
        for (uint32_t r = 0; r < R; ++r) D |= (D << 1) & A;
        if (D & F) return 1;
        if (!D && !Iall) return 0;
    }
    return (D & Fe) != 0;
}

}  // namespace

extern "C" {

int bt_payload_dfa_compile(const char* expression, void* blob, uint32_t cap, uint32_t* size) {
    return bt_payload_dfa_compile_ex(expression, 0, blob, cap, size);
}

int bt_payload_dfa_compile_ex(const char* expression, uint32_t flags, void* blob, uint32_t cap, uint32_t* size) {
    if (!expression || !size) return BT_E_INVALID_ARGUMENT;
    const std::string e(expression);
    try {
        std::regex probe(e);   // the reference's own acceptance (src/PacketFilter.cpp:311-316)
    } catch (const std::regex_error&) {
        return BT_E_INVALID_ARGUMENT;
    }
    if (!(flags & BT_DFA_NO_BITPAR)) {   // the bit-parallel form where the pattern fits it
        try {
            const BitparBlob o = build_bitpar(e);
            *size = bitpar_size(o);
            if (!blob) return BT_OK;
            if (cap < *size) return BT_E_RESOURCE;
            bitpar_write(o, static_cast<uint8_t*>(blob));
            return BT_OK;
        } catch (const Unsupported&) {
        }
    }
    Packed pk;
    try {
        pk = pack(build_dfa(e), !(flags & BT_DFA_NO_PAIRS));
    } catch (const Unsupported&) {
        return BT_E_NOT_IMPLEMENTED;
    }
    *size = blob_size(pk);
    if (!blob) return BT_OK;
    if (cap < *size) return BT_E_RESOURCE;
    uint8_t* p = static_cast<uint8_t*>(blob);
    std::memset(p, 0, *size);
    const uint16_t k16 = (uint16_t)pk.K, c16 = (uint16_t)pk.C;
    std::memcpy(p, &k16, 2);
    std::memcpy(p + 2, &c16, 2);
    p[4] = (uint8_t)pk.init;
    p[5] = (uint8_t)pk.empty;
    p[6] = pk.P ? 1 : 0;
    p[7] = (uint8_t)pk.P;
    uint8_t* q = p + 8;
    if (pk.K) std::memcpy(q, pk.endacc.data(), pk.K);
    q += (pk.K + 3) & ~3;
    if (pk.C != 256) {
        std::memcpy(q, pk.cls.data(), 256);
        q += 256;
    }
    if (!pk.next.empty()) std::memcpy(q, pk.next.data(), pk.next.size());
    q += pk.next.size();
    if (pk.P) {
        q = p + (((size_t)(q - p) + 3) & ~(size_t)3);
        std::memcpy(q, pk.clsp.data(), 256);
        std::memcpy(q + 256, pk.pair.data(), pk.pair.size());
    }
    return BT_OK;
}

int bt_payload_dfa_search(const void* blob, const uint8_t* s, uint32_t n) {
    const uint8_t* p = static_cast<const uint8_t*>(blob);
    uint16_t K, C;
    std::memcpy(&K, p, 2);
    if (K == kBitparMagic) return bitpar_search(p, s, n);
    std::memcpy(&C, p + 2, 2);
    const uint8_t* endacc = p + 8;
    const uint8_t* cls = endacc + ((K + 3) & ~3);
    const uint8_t* next = C == 256 ? cls : cls + 256;
    uint32_t q = p[4];
    if (n == 0) return p[5];
    if (q >= K) return q == K;
    uint32_t i = 0;
    if (p[6]) {   // two bytes per dependent step, as the kernel walks it
        const uint32_t P = p[7];
        const size_t at = ((size_t)(next + (size_t)K * C - p) + 3) & ~(size_t)3;
        const uint8_t* clsp = p + at;
        const uint8_t* pair = clsp + 256;
        for (; i + 2 <= n; i += 2) {
            q = pair[(q * P + clsp[s[i]]) * P + clsp[s[i + 1]]];
            if (q >= K) return q == K;
        }
    }
    for (; i < n; ++i) {
        q = next[q * C + (C == 256 ? s[i] : cls[s[i]])];
        if (q >= K) return q == K;
    }
    return endacc[q];
}

int bt_payload_dfa_eval(const void* blob, const uint8_t* frame, uint32_t len) {
    // applyPayloadFilter's window (src/PacketFilter.cpp:293-309)
    if (len < 34) return 0;
    if (((uint32_t)frame[12] << 8 | frame[13]) != 0x0800u) return 0;
    const uint32_t off = 14 + (uint32_t)(frame[14] & 0x0F) * 4;
    if (len <= off) return 0;
    return bt_payload_dfa_search(blob, frame + off, std::min<uint32_t>(len - off, 100));
}

}  // extern "C"
