// Drives include/aloam_lidar_factor.hpp (the lidarFactor.hpp API mirror) on factor records read
// from stdin and prints the residuals: tests/test_lidar_factor_api.py compares them with the
// oracle's Jet evaluation and checks to_device() round trips the record.
#include <cstdio>
#include <cstring>
#include <initializer_list>

#include "../include/aloam_lidar_factor.hpp"

int main() {
    double x[7];
    for (double& v : x) if (scanf("%lf", &v) != 1) return 2;
    int n;
    if (scanf("%d", &n) != 1) return 2;
    for (int i = 0; i < n; i++) {
        int type;
        double cp[3], a[3], b[3], c[3];
        if (scanf("%d", &type) != 1) return 2;
        for (double* v : {cp, a, b, c}) for (int k = 0; k < 3; k++) if (scanf("%lf", &v[k]) != 1) return 2;
        double r[3] = {0, 0, 0};
        aloam_factor f;
        bool ok = false;
        if (type == 0) { LidarEdgeFactor e(cp, a, b, 1.0); e(x, x + 4, r); ok = e.to_device(&f); }
        else if (type == 1) { LidarPlaneFactor p(cp, a, b, c, 1.0); p(x, x + 4, r); ok = p.to_device(&f);
                              printf("N %.17g %.17g %.17g\n", p.ljm_norm[0], p.ljm_norm[1], p.ljm_norm[2]); }
        else if (type == 2) { LidarPlaneNormFactor p(cp, a, b[0]); p(x, x + 4, r); ok = p.to_device(&f); }
        else { LidarDistanceFactor d(cp, a); d(x, x + 4, r); ok = d.to_device(&f); }
        printf("R %d %.17g %.17g %.17g %d\n", f.type, r[0], r[1], r[2], ok ? 1 : 0);
    }
    return 0;
}
