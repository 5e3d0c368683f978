// oracle/_ref/ref_jsf: the reference's own jsf32 (3rd/rng/jsf.h, header-only, compiled in
// place with -I; never copied) printing its first N draws from the default seed, the
// sequence AbstractMetricsManager's deep sampling uses (src/AbstractMetricsManager.h:245,321).
// Test infrastructure: pins the restatements in pv_host.cpp and pv_oracle.cpp.
#include <cstdio>
#include <cstdlib>

#include <jsf.h>

int main(int argc, char **argv)
{
    const long n = argc > 1 ? atol(argv[1]) : 16;
    jsf32 r;
    for (long i = 0; i < n; i++) printf("%u\n", (unsigned)r());
    return 0;
}
