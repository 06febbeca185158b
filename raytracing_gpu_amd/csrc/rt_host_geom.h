// rt_host_geom.h — host-side primitive bounding boxes (sphere.h:75-78, moving_sphere.h:61-66,
// aarect.h bounding_box, triangle.h:46-98), shared by the scene library and rt_scene_upload.
#pragma once

#include <algorithm>
#include <cmath>

#include "../../include/rt_hip.h"

namespace rth {

struct Box {
  float lo[3], hi[3];
};

inline Box join(const Box& a, const Box& b) {
  Box r;
  for (int k = 0; k < 3; ++k) {
    r.lo[k] = std::fmin(a.lo[k], b.lo[k]);
    r.hi[k] = std::fmax(a.hi[k], b.hi[k]);
  }
  return r;
}

// bounding_box(t0, t1) of prim q, with the reference's float rounding.
inline Box prim_box(const rt_prim& q, const rt_triangle* tris, float t0, float t1) {
  const float* p = q.p;
  Box b;
  switch (q.type & 0xff) {
    case RT_PRIM_SPHERE:
      for (int k = 0; k < 3; ++k) {
        b.lo[k] = p[k] - p[3];
        b.hi[k] = p[k] + p[3];
      }
      return b;
    case RT_PRIM_MOVING_SPHERE: {
      Box a, c;
      const float sa = (t0 - p[7]) / p[8], sb = (t1 - p[7]) / p[8];
      for (int k = 0; k < 3; ++k) {
        const float ca = p[k] + sa * p[4 + k], cb = p[k] + sb * p[4 + k];
        a.lo[k] = ca - p[3];
        a.hi[k] = ca + p[3];
        c.lo[k] = cb - p[3];
        c.hi[k] = cb + p[3];
      }
      return join(a, c);
    }
    case RT_PRIM_RECT_XY:
      return Box{{p[0], p[2], p[4] - 0.0001f}, {p[1], p[3], p[4] + 0.0001f}};
    case RT_PRIM_RECT_XZ:  // xz_rect uses z1 for both z bounds (aarect.h:39, H4)
      return Box{{p[0], p[4] - 0.0001f, p[3]}, {p[1], p[4] + 0.0001f, p[3]}};
    case RT_PRIM_RECT_YZ:
      return Box{{p[4] - 0.0001f, p[0], p[2]}, {p[4] + 0.0001f, p[1], p[3]}};
    case RT_PRIM_BOX:  // box.h:35-38
      return Box{{p[0], p[1], p[2]}, {p[3], p[4], p[5]}};
    default: {
      const rt_triangle& t = tris[(int)p[0]];
      float v[3][3];
      for (int k = 0; k < 3; ++k) {
        v[0][k] = t.v0[k];
        v[1][k] = t.v1[k];
        v[2][k] = t.v2[k];
      }
      for (int k = 0; k < 3; ++k) {
        b.lo[k] = std::min({v[0][k], v[1][k], v[2][k]});
        b.hi[k] = std::max({v[0][k], v[1][k], v[2][k]});
        if (std::fabs(b.lo[k] - b.hi[k]) < 0.000001f) {  // triangle.h:84-95 padding
          b.hi[k] += 0.0001f;
          b.lo[k] -= 0.0001f;
        }
      }
      return b;
    }
  }
}

}  // namespace rth
