// CPU check of the light-hierarchy depth guard (host/light_select.cpp, compiled
// here with g++): lights at geometrically shrinking positions make the
// insertion-built PointBvh one level deeper per light.  Up to 32 levels the
// hierarchy selector is kept; deeper trees, whose left/right codes would need
// more than 32 bits, get the flux CDF ("simple") selector instead.
#include "light_select.h"

#include <cstdio>
#include <vector>

static std::vector<igx_light> geometric(int n) {
    std::vector<igx_light> v(n);
    for (int i = 0; i < n; ++i) {
        igx_light L{};
        L.type = IGX_LIGHT_POINT;
        float x = 1.0f;
        for (int k = 0; k < i; ++k) x *= 0.5f;
        L.select_position[0] = x;
        L.select_flux = 1.0f + (float)i;
        v[i] = L;
    }
    return v;
}

int main() {
    int bad = 0;
    for (int n : {8, 30, 40, 64}) {
        const auto lights = geometric(n);
        const igx::LightSelectTables t = igx::build_light_select(IGX_SELECT_HIERARCHY, n, lights);
        std::printf("lights %d selector %d cdf %zu hierarchy %zu\n", n, t.selector, t.cdf.size(), t.hierarchy.size());
        const int want = n <= 32 ? IGX_SELECT_HIERARCHY : IGX_SELECT_SIMPLE;
        if (t.selector != want) {
            std::printf("FAIL: %d lights: selector %d, want %d\n", n, t.selector, want);
            ++bad;
        }
        if (t.selector == IGX_SELECT_SIMPLE && (t.cdf.size() != (size_t)n || t.cdf.back() != 1.0f)) {
            std::printf("FAIL: %d lights: bad CDF\n", n);
            ++bad;
        }
    }
    std::printf(bad ? "failed\n" : "ok\n");
    return bad ? 1 : 0;
}
