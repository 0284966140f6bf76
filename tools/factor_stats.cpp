// factor_stats.cpp — host-only analysis of a regex signature set's prefilter plan (design
// probe for the C4 prefilter): factor length histogram, patterns per
// factor, patterns without a factor set. Reads the set as <u32 count><u32 len><bytes>...
// Build: g++ -O2 -std=c++17 tools/factor_stats.cpp swarm_amd/csrc/sg_regex.cpp -o tools/bin/factor_stats
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <map>
#include <vector>
#include "../swarm_amd/csrc/sg_regex.hpp"

namespace sg {
void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    fputc('\n', stderr);
    va_end(ap);
}
}  // namespace sg

int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    uint32_t n = 0;
    if (fread(&n, 4, 1, f) != 1) return 1;
    std::vector<uint8_t> blob;
    std::vector<uint32_t> offs(1, 0);
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t l = 0;
        if (fread(&l, 4, 1, f) != 1) return 1;
        size_t o = blob.size();
        blob.resize(o + l);
        if (l && fread(blob.data() + o, 1, l, f) != l) return 1;
        offs.push_back((uint32_t)blob.size());
    }
    fclose(f);
    sg::RegexPlan plan;
    int rc = sg::regex_build_plan(blob.data(), offs.data(), n, 0, &plan);
    if (rc) { fprintf(stderr, "plan rc %d\n", rc); return 2; }
    std::map<size_t, uint32_t> lenh;
    std::map<size_t, uint32_t> lenp;  // patterns reachable through factors of that length
    for (size_t k = 0; k < plan.factors.size(); ++k) {
        const size_t L = plan.factors[k].size();
        lenh[L]++;
        lenp[L] += plan.fac_off[k + 1] - plan.fac_off[k];
    }
    printf("patterns %u, filtered %zu, unfiltered groups %zu, factors %zu\n", n, plan.singles.size(), plan.groups.size(),
           plan.factors.size());
    uint32_t grp_states = 0;
    for (auto &g : plan.groups) grp_states += g.n_states;
    printf("factor-less group states %u\n", grp_states);
    for (auto &kv : lenh) printf("factor len %2zu: %5u factors, %6u (factor, pattern) pairs\n", kv.first, kv.second, lenp[kv.first]);
    // the most shared factors
    std::vector<std::pair<uint32_t, size_t>> sh;
    for (size_t k = 0; k < plan.factors.size(); ++k) sh.push_back({plan.fac_off[k + 1] - plan.fac_off[k], k});
    std::sort(sh.rbegin(), sh.rend());
    for (size_t i = 0; i < sh.size() && i < 25; ++i)
        printf("  shared by %4u: '%.*s'\n", sh[i].first, (int)plan.factors[sh[i].second].size(),
               (const char *)plan.factors[sh[i].second].data());
    // short factors
    int shown = 0;
    for (size_t k = 0; k < plan.factors.size() && shown < 40; ++k)
        if (plan.factors[k].size() == 3) {
            printf("  3-byte: '%.*s' x%u\n", 3, (const char *)plan.factors[k].data(), plan.fac_off[k + 1] - plan.fac_off[k]);
            ++shown;
        }
    return 0;
}
