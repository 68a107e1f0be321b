// test_regex_dfa.cpp — the PAYLOAD DFA compiler (beatrice_amd/csrc/bt_regex_dfa.cpp)
// against std::regex_search, the function the reference's applyPayloadFilter calls
// (src/PacketFilter.cpp:311-313; libstdc++ <regex>, ECMAScript, default flags).
//
//   test_regex_dfa [patterns] [strings_per_pattern] [seed]
//
// 1. A fixed list of realistic and corner-case patterns.
// 2. Random patterns from a grammar over the modelled subset (literals incl. \n \r NUL
//    and bytes >= 0x80, ., classes with ranges / negation / escapes, \d\w\s, groups,
//    alternation, all quantifiers incl. stacked and lazy, ^ $ anywhere).
// Every pattern std::regex accepts is compiled twice, in the form the compiler prefers (the
// bit-parallel Shift-And form where the pattern is a union of linear class sequences, else
// the DFA) and as a DFA (BT_DFA_NO_BITPAR); where the compiler takes it (not
// BT_E_NOT_IMPLEMENTED) each blob must agree with regex_search on every test string:
// random strings over an alphabet that hits every class boundary, lengths 0..40,
// plus the full applyPayloadFilter window path on synthetic frames.
// libstdc++'s regex_search backtracks (exponential on nested quantifiers), so each
// random pattern is checked in a forked child under a 2 s alarm; patterns std::regex
// itself cannot finish are counted and skipped. Exit status 0 = no disagreement. CPU only.
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <regex>
#include <string>
#include <vector>

#include "beatrice_gpu_bench.h"

extern "C" int bt_payload_dfa_compile(const char* expression, void* blob, uint32_t cap, uint32_t* size);
extern "C" int bt_payload_dfa_compile_ex(const char* expression, uint32_t flags, void* blob, uint32_t cap,
                                         uint32_t* size);
extern "C" int bt_payload_dfa_search(const void* blob, const uint8_t* s, uint32_t n);
extern "C" int bt_payload_dfa_eval(const void* blob, const uint8_t* frame, uint32_t len);

static const char kAlpha[] = {'a', 'b', 'c', 'A', 'Z', '0', '9', '_', '-', ' ', '\t', '\n', '\r', '\v', '\0',
                              '.', '/', ']', '}', '^', '$', '\\', (char)0x7f, (char)0x80, (char)0xc3, (char)0xff,
                              'G', 'E', 'T', 'x'};

struct Gen {
    std::mt19937_64 r;
    explicit Gen(uint64_t s) : r(s) {}
    int pick(int n) { return (int)(r() % (uint64_t)n); }

    std::string lit() {
        static const char* L[] = {"a", "b", "c", "G", "E", "T", "x", "0", "9", "_", "-", " ", "/", "]", "}",
                                  "\\.", "\\-", "\\/", "\\\\", "\\t", "\\n", "\\r", "\\x00", "\\x80", "\\xff",
                                  "\\x41", "\\0", "\\$", "\\^", "\\[", "\\(", "\\*", "\\?"};
        return L[pick(sizeof(L) / sizeof(L[0]))];
    }
    std::string cls() {
        static const char* C[] = {"[abc]", "[^a]", "[a-c]", "[a-]", "[-a]", "[^-]", "[\\d]", "[\\w-]", "[\\s]",
                                  "[^\\W]", "[\\]a]", "[\\b]", "[\\x80-\\xff]", "[\\x00-\\x20]", "[A-Za-z0-9]",
                                  "[]", "[^]", "[.]", "[$^]", "[\\n\\r]", "[^\\n]", "[a-c\\d]", "[\\x80-\\x10]"};
        return C[pick(sizeof(C) / sizeof(C[0]))];
    }
    std::string atom(int depth) {
        switch (pick(depth > 2 ? 5 : 7)) {
        case 0: case 1: return lit();
        case 2: return ".";
        case 3: return cls();
        case 4: {
            static const char* E[] = {"\\d", "\\D", "\\w", "\\W", "\\s", "\\S"};
            return E[pick(6)];
        }
        case 5: return "(" + re(depth + 1) + ")";
        default: return "(?:" + re(depth + 1) + ")";
        }
    }
    std::string quant() {
        static const char* Q[] = {"", "", "", "*", "+", "?", "{2}", "{0,2}", "{1,}", "*?", "+?", "??", "{0}", "**",
                                  "{2,3}", "{3}"};
        return Q[pick(sizeof(Q) / sizeof(Q[0]))];
    }
    std::string term(int depth) {
        const int k = pick(12);
        if (k == 0) return "^";
        if (k == 1) return "$";
        return atom(depth) + quant();
    }
    std::string re(int depth = 0) {
        std::string s;
        const int n = 1 + pick(4);
        for (int i = 0; i < n; ++i) s += term(depth);
        if (pick(4) == 0) s += "|" + (pick(3) ? re(depth + 1) : std::string());
        return s;
    }
    std::string str() {
        const int n = pick(41);
        std::string s;
        for (int i = 0; i < n; ++i) s += kAlpha[pick(sizeof(kAlpha))];
        return s;
    }
};

static int g_bad = 0, g_checked = 0, g_unsupported = 0, g_rejected = 0, g_slow = 0, g_bitpar = 0;

static bool check_form(const std::string& pat, const std::regex& re, Gen& g, int nstr, uint32_t flags);

static bool check(const std::string& pat, Gen& g, int nstr) {
    std::regex re;
    try {
        re = std::regex(pat);
    } catch (const std::regex_error&) {
        ++g_rejected;
        uint32_t sz = 0;
        if (bt_payload_dfa_compile(pat.c_str(), nullptr, 0, &sz) != BT_E_INVALID_ARGUMENT) {
            std::printf("FAIL pattern std::regex rejects was not rejected: /%s/\n", pat.c_str());
            ++g_bad;
            return false;
        }
        return true;
    }
    uint32_t sz = 0;
    const int rc = bt_payload_dfa_compile(pat.c_str(), nullptr, 0, &sz);
    if (rc == BT_E_NOT_IMPLEMENTED) {
        ++g_unsupported;
        return true;
    }
    if (rc != BT_OK) {
        std::printf("FAIL compile rc %d for /%s/\n", rc, pat.c_str());
        ++g_bad;
        return false;
    }
    ++g_checked;
    // the preferred form, then the DFA of the same pattern (the same strings: a copy of g)
    Gen g2 = g;
    if (!check_form(pat, re, g, nstr, 0)) return false;
    if (bt_payload_dfa_compile(pat.c_str(), nullptr, 0, &sz) == BT_OK) {
        std::vector<uint8_t> b(sz);
        bt_payload_dfa_compile(pat.c_str(), b.data(), sz, &sz);
        if (b[0] == 0xFF && b[1] == 0xFF) {
            ++g_bitpar;
            uint32_t s2 = 0;
            if (bt_payload_dfa_compile_ex(pat.c_str(), BT_DFA_NO_BITPAR, nullptr, 0, &s2) == BT_OK)
                return check_form(pat, re, g2, nstr, BT_DFA_NO_BITPAR);
        }
    }
    return true;
}

static bool check_form(const std::string& pat, const std::regex& re, Gen& g, int nstr, uint32_t flags) {
    uint32_t sz = 0;
    bt_payload_dfa_compile_ex(pat.c_str(), flags, nullptr, 0, &sz);
    std::vector<uint8_t> blob(sz);
    bt_payload_dfa_compile_ex(pat.c_str(), flags, blob.data(), sz, &sz);
    const char* form = blob.size() >= 2 && blob[0] == 0xFF && blob[1] == 0xFF ? "bitpar" : "dfa";
    for (int k = 0; k < nstr; ++k) {
        const std::string s = k == 0 ? std::string() : g.str();
        bool want;
        try {
            want = std::regex_search(s, re);
        } catch (const std::regex_error&) {
            continue;   // complexity / stack errors: the reference returns false; not modelled
        }
        const int got = bt_payload_dfa_search(blob.data(), reinterpret_cast<const uint8_t*>(s.data()), (uint32_t)s.size());
        if (got != (int)want) {
            std::string hex;
            for (unsigned char c : s) {
                char b[4];
                std::snprintf(b, sizeof(b), "%02x", c);
                hex += b;
            }
            std::printf("FAIL /%s/ on [%s] (len %zu): std::regex %d %s %d\n", pat.c_str(), hex.c_str(), s.size(), want,
                        form, got);
            ++g_bad;
            return false;
        }
    }
    // the applyPayloadFilter window on frames: IPv4 header of IHL 5..15, payload after it
    for (int k = 0; k < 20; ++k) {
        std::vector<uint8_t> f(14 + 60 + 120, 0);
        f[12] = 0x08;
        f[13] = k == 3 ? 0x06 : 0x00;   // one non-IPv4 frame
        const int ihl = 5 + g.pick(11);
        f[14] = (uint8_t)(0x40 | ihl);
        const std::string s = g.str() + g.str() + g.str() + g.str();
        const size_t off = 14 + 4 * ihl;
        for (size_t i = 0; i < s.size() && off + i < f.size(); ++i) f[off + i] = (uint8_t)s[i];
        const uint32_t len = (uint32_t)std::min(f.size(), off + (size_t)g.pick(130));
        bool want = false;
        if (len >= 34 && f[12] == 0x08 && f[13] == 0x00 && len > off) {
            std::string pay(reinterpret_cast<const char*>(f.data() + off), std::min<size_t>(len - off, 100));
            try {
                want = std::regex_search(pay, re);
            } catch (const std::regex_error&) {
                continue;
            }
        }
        if (bt_payload_dfa_eval(blob.data(), f.data(), len) != (int)want) {
            std::printf("FAIL /%s/ %s frame eval (ihl %d len %u)\n", pat.c_str(), form, ihl, len);
            ++g_bad;
            return false;
        }
    }
    return true;
}

int main(int argc, char** argv) {
    const int npat = argc > 1 ? std::atoi(argv[1]) : 3000;
    const int nstr = argc > 2 ? std::atoi(argv[2]) : 200;
    Gen g(argc > 3 ? std::strtoull(argv[3], nullptr, 0) : 12345);
    const char* fixed[] = {"GET", "GET|POST", "HTTP/1\\.[01]", "^GET /", "User-Agent: .*bot", "[A-Z]{3,} /",
                           "(POST|PUT) /api", "\\d{3}-\\d{4}", "\\s+$", "^$", "a|", "()", "[^]", "[]", "x*",
                           "^\\x16\\x03[\\x00-\\x03]", "beatrice", "[", "a{2,1}", "\\1", "(a)\\1", "\\bfoo",
                           "(?=a)b", "[[:alpha:]]", "\\cA", "\\u0041", "a^b", "a$b", "$^", "^^a$$", "(a|b)*abb",
                           "(a|ab)(c|bcd)(d*)", "[\\x80-\\xff]+", ".{100}", "a{0}b", "\\x00\\x01", "\\0"};
    for (const char* p : fixed) check(p, g, nstr);
    for (int i = 0; i < npat; ++i) {
        const std::string pat = g.re();
        const uint64_t seed = g.r();
        fflush(stdout);
        const pid_t pid = fork();
        if (pid == 0) {
            alarm(2);
            Gen gc(seed);
            g_bad = g_checked = g_unsupported = g_rejected = g_bitpar = 0;
            check(pat, gc, nstr);
            fflush(stdout);
            _exit(g_bad ? 1 : g_bitpar ? 5 : g_checked ? 4 : g_unsupported ? 2 : 3);
        }
        int st = 0;
        waitpid(pid, &st, 0);
        if (WIFSIGNALED(st)) {
            ++g_slow;
            continue;
        }
        switch (WEXITSTATUS(st)) {
        case 1: ++g_bad; break;
        case 2: ++g_unsupported; break;
        case 3: ++g_rejected; break;
        case 5: ++g_checked; ++g_bitpar; break;
        default: ++g_checked; break;
        }
    }
    std::printf("patterns: %d compiled and checked (%d of them in the bit-parallel form, checked as a DFA too), "
                "%d left on the host (outside the subset), %d rejected by std::regex, %d skipped "
                "(std::regex_search > 2 s); %d disagreements\n",
                g_checked, g_bitpar, g_unsupported, g_rejected, g_slow, g_bad);
    if (g_bad) {
        std::printf("%d FAILED\n", g_bad);
        return 1;
    }
    std::printf("ALL OK\n");
    return 0;
}
