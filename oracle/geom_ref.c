/* ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
 *
 * Plain-C restatement of the reference's integer pillar index
 * (reference model/bev_model.py:45-57 get_geometry, :85-95 voxelisation/mask/rank):
 *   p    = (u*d, v*d, d)                                     frustum point (fp32)
 *   xyz  = ((c0*p0 + c1*p1) + c2*p2) + t                     per row, sequential fp32, no FMA
 *   g    = trunc((xyz - lo) / res)                           Tensor.long() truncates toward 0
 *   rank = gx*Y*Z + gy*Z + gz if 0<=g<dim on all axes else -1
 * Compiled with -ffp-contract=off so every multiply and add rounds separately, matching the
 * reference's fp32 CPU matmul bit for bit (checked against tests/golden/geometry_*.npz).
 */
#include <math.h>
#include <stdint.h>

void oracle_geom_index(const float *frustum, const float *combine, const float *trans,
                       const float *lo, const float *res, int X, int Y, int Z, int B, int N,
                       int D, int h, int w, int32_t *pillar, float *xyz_out) {
  const long dhw = (long)D * h * w;
  for (long bn = 0; bn < (long)B * N; ++bn) {
    const float *c = combine + 9 * bn, *t = trans + 3 * bn;
    for (long f = 0; f < dhw; ++f) {
      const float u = frustum[3 * f], v = frustum[3 * f + 1], d = frustum[3 * f + 2];
      const float p[3] = {u * d, v * d, d};
      float g[3];
      for (int r = 0; r < 3; ++r) {
        float a = c[3 * r] * p[0];
        a = a + c[3 * r + 1] * p[1];
        a = a + c[3 * r + 2] * p[2];
        a = a + t[r];
        if (xyz_out) xyz_out[(bn * dhw + f) * 3 + r] = a;
        g[r] = truncf((a - lo[r]) / res[r]);
      }
      const int ok = g[0] >= 0.f && g[0] < (float)X && g[1] >= 0.f && g[1] < (float)Y &&
                     g[2] >= 0.f && g[2] < (float)Z;
      pillar[bn * dhw + f] = ok ? (int32_t)g[0] * Y * Z + (int32_t)g[1] * Z + (int32_t)g[2] : -1;
    }
  }
}
