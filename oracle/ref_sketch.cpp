// oracle/ref_sketch.cpp — TEST INFRASTRUCTURE ONLY.
// Drives the reference's vendored datasketches (3rd/datasketches, compiled in
// place by oracle/Makefile into oracle/_ref/ref_sketch) so that the oracle's
// restated CPC HIP/ICON estimator and exact-mode KLL rank rule can be pinned to
// the real library. Protocol (stdin, one command per line):
//   cpc_u32 <merged 0|1> <n> v1 v2 ...      -> prints the estimate (%.17g)
//   cpc_str <merged 0|1> <n> s1 s2 ...      -> idem, string items (no spaces)
//   kll_u64 <n> v1 ... vn                   -> prints p50 p90 p95 p99
//   fi_str  <n> s1 ... sn                   -> prints "item:estimate" sorted as the library returns
#include <cpc_sketch.hpp>
#include <cpc_union.hpp>
#include <frequent_items_sketch.hpp>
#include <kll_sketch.hpp>
#include <cstdio>
#include <iostream>
#include <string>
#include <vector>

int main()
{
    std::string cmd;
    while (std::cin >> cmd) {
        if (cmd == "cpc_u32" || cmd == "cpc_str") {
            int merged; size_t n;
            std::cin >> merged >> n;
            datasketches::cpc_sketch s(11);
            for (size_t i = 0; i < n; i++) {
                if (cmd == "cpc_u32") { uint32_t v; std::cin >> v; s.update(v); }
                else { std::string v; std::cin >> v; s.update(v); }
            }
            double est;
            if (merged) {
                datasketches::cpc_union u(11);
                u.update(s);
                est = u.get_result().get_estimate();
            } else est = s.get_estimate();
            printf("%.17g\n", est);
        } else if (cmd == "kll_u64") {
            size_t n; std::cin >> n;
            datasketches::kll_sketch<uint64_t> k;
            for (size_t i = 0; i < n; i++) { uint64_t v; std::cin >> v; k.update(v); }
            printf("%llu %llu %llu %llu\n", (unsigned long long)k.get_quantile(0.5), (unsigned long long)k.get_quantile(0.9),
                (unsigned long long)k.get_quantile(0.95), (unsigned long long)k.get_quantile(0.99));
        } else if (cmd == "fi_str") {
            size_t n; std::cin >> n;
            datasketches::frequent_items_sketch<std::string> fi(13, 7);
            for (size_t i = 0; i < n; i++) { std::string v; std::cin >> v; fi.update(v); }
            auto items = fi.get_frequent_items(datasketches::frequent_items_error_type::NO_FALSE_NEGATIVES);
            printf("maxerr %llu", (unsigned long long)fi.get_maximum_error());
            for (auto &r : items) printf(" %s:%llu", r.get_item().c_str(), (unsigned long long)r.get_estimate());
            printf("\n");
        }
        fflush(stdout);
    }
    return 0;
}
