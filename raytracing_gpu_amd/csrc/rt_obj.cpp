// rt_obj.cpp — OBJ mesh ingestion for the mesh scenes (door, cup): the host side of
// create_meshes() (triangle_mesh.h:208-352).
//
// The reference reads meshes with assimp (Importer::ReadFile(path, Triangulate | GenNormals),
// triangle_mesh.h:129-143) and walks the node tree (processNode/processMesh, :51-126), then builds
// one triangle per 3 indices in create_meshes_d (:147-204).  Assimp is not available here, so this
// file restates the parts of assimp's OBJ import that decide the triangles:
//   * number parsing: fast_atoreal_move (integer part as float, plus the fraction rounded from
//     double: two roundings, not strtof);
//   * one aiMesh per (object, material) run, in file order; the root node's children are the
//     objects in order, each holding its meshes in order;
//   * every polygon corner is its own vertex (no sharing across polygons);
//   * Triangulate: triangles unchanged; quads fanned from their concave corner (or corner 0);
//     larger polygons ear-clipped in the 2D projection picked by the Newell normal, then triangles
//     whose projected area is below 1e-5 dropped;
//   * GenNormals (only when the file has no normals): per-face normals, later faces overwrite
//     shared corners.
// Pinned against assimp (v3.3, the build embedded in this container's Qt3D scene-import plugin)
// by tests/golden/make_obj_golden.py; the reference used assimp 5.x.
//
// create_meshes_d indexes the concatenated vertex array with each mesh's local indices (no offset
// for the first file); RT_OBJ_INDEX_REFERENCE keeps that, RT_OBJ_INDEX_GLOBAL adds
// each mesh's vertex offset (the evident intent).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"

namespace {

struct P3 {
  float x, y, z;
  float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
struct P2 {
  float x, y;
};

// fast_atoreal_move<float> of assimp's fast_atof.h.
float atof_assimp(const char* c) {
  const bool inv = *c == '-';
  if (inv || *c == '+') ++c;
  float f = 0.0f;
  if (*c != '.') {
    uint64_t v = 0;
    while (*c >= '0' && *c <= '9') v = v * 10 + (uint64_t)(*c++ - '0');
    f = (float)v;
  }
  if (*c == '.' && c[1] >= '0' && c[1] <= '9') {
    ++c;
    uint64_t v = 0;
    int digits = 0;
    while (*c >= '0' && *c <= '9') {
      if (digits < 15) {
        v = v * 10 + (uint64_t)(*c - '0');
        ++digits;
      }
      ++c;
    }
    double pl = (double)v;
    static const double table[16] = {0.0,   0.1,   0.01,   0.001,   0.0001,   0.00001,   0.000001,   0.0000001,
                                      1e-8, 1e-9, 1e-10, 1e-11, 1e-12, 1e-13, 1e-14, 1e-15};
    pl *= table[digits];
    f += (float)pl;
  } else if (*c == '.') {
    ++c;
  }
  if (*c == 'e' || *c == 'E') {
    ++c;
    const bool einv = *c == '-';
    if (einv || *c == '+') ++c;
    uint64_t e = 0;
    while (*c >= '0' && *c <= '9') e = e * 10 + (uint64_t)(*c++ - '0');
    float ex = (float)e;
    if (einv) ex = -ex;
    f *= std::pow(10.0f, ex);
  }
  return inv ? -f : f;
}

struct Corner {
  int v, t, n;  // 0-based, -1 = absent
};
constexpr int kNoMaterial = -1;
struct Mesh {
  int material = kNoMaterial;  // index into the material library, 0 = assimp's default material
  std::vector<std::vector<Corner>> faces;
};
struct Object {
  std::string name;
  std::vector<int> meshes;
};

// 2D helpers of assimp's PolyTools.h (float arithmetic).
inline float area2d(const P2& a, const P2& b, const P2& c) {
  return 0.5f * (a.x * (c.y - b.y) + b.x * (a.y - c.y) + c.x * (b.y - a.y));
}
inline bool on_left(const P2& p0, const P2& p1, const P2& p2) { return area2d(p0, p2, p1) > 0.0f; }
inline bool in_tri(const P2& p0, const P2& p1, const P2& p2, const P2& pp) {
  const P2 v0{p1.x - p0.x, p1.y - p0.y}, v1{p2.x - p0.x, p2.y - p0.y}, v2{pp.x - p0.x, pp.y - p0.y};
  double d00 = v0.x * v0.x + v0.y * v0.y;
  const double d01 = v0.x * v1.x + v0.y * v1.y;
  const double d02 = v0.x * v2.x + v0.y * v2.y;
  double d11 = v1.x * v1.x + v1.y * v1.y;
  const double d12 = v1.x * v2.x + v1.y * v2.y;
  const double inv = 1 / (d00 * d11 - d01 * d01);
  d11 = (d11 * d02 - d01 * d12) * inv;
  d00 = (d00 * d12 - d01 * d02) * inv;
  return (d11 > 0) && (d00 > 0) && (d11 + d00 < 1);
}

// Triangulate one polygon of n >= 4 corners whose vertices are pos[0..n) (mesh-local indices
// base..base+n); appends index triples.
void triangulate(const std::vector<P3>& pos, unsigned base, std::vector<unsigned>& out) {
  const int n = (int)pos.size();
  if (n == 4) {  // quads: fan from the concave corner, if any
    int start = 0;
    for (int i = 0; i < 4; ++i) {
      const P3 &v0 = pos[(i + 3) % 4], &v1 = pos[(i + 2) % 4], &v2 = pos[(i + 1) % 4], &v = pos[i];
      P3 l{v0.x - v.x, v0.y - v.y, v0.z - v.z}, d{v1.x - v.x, v1.y - v.y, v1.z - v.z},
          r{v2.x - v.x, v2.y - v.y, v2.z - v.z};
      auto norm = [](P3& a) {  // aiVector3D::Normalize: *this /= Length()
        const float len = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
        a.x /= len;
        a.y /= len;
        a.z /= len;
      };
      norm(l);
      norm(d);
      norm(r);
      const float angle = std::acos(l.x * d.x + l.y * d.y + l.z * d.z) + std::acos(r.x * d.x + r.y * d.y + r.z * d.z);
      if (angle > 3.14159265358979323846f) {
        start = i;
        break;
      }
    }
    const unsigned t[4] = {base, base + 1, base + 2, base + 3};
    out.insert(out.end(), {t[start], t[(start + 1) % 4], t[(start + 2) % 4]});
    out.insert(out.end(), {t[start], t[(start + 2) % 4], t[(start + 3) % 4]});
    return;
  }
  // Newell normal (float sums), projection axes
  float sxy = 0.0f, syz = 0.0f, szx = 0.0f;
  for (int k = 0; k < n; ++k) {
    const P3 &p = pos[(k + 1) % n], &lo = pos[k], &hi = pos[(k + 2) % n];
    sxy += p.x * (hi.y - lo.y);
    syz += p.y * (hi.z - lo.z);
    szx += p.z * (hi.x - lo.x);
  }
  const P3 nn{syz, szx, sxy};
  const float ax = std::fabs(nn.x), ay = std::fabs(nn.y), az = std::fabs(nn.z);
  int ac = 0, bc = 1;
  float inv = nn.z;
  if (ax > ay) {
    if (ax > az) {
      ac = 1;
      bc = 2;
      inv = nn.x;
    }
  } else if (ay > az) {
    ac = 2;
    bc = 0;
    inv = nn.y;
  }
  if (inv < 0.0f) std::swap(ac, bc);
  std::vector<P2> tv(n);
  std::vector<char> done(n, 0);
  for (int k = 0; k < n; ++k) tv[k] = P2{pos[k][ac], pos[k][bc]};
  std::vector<int> tri;  // local corner triples
  int num = n, ear = 0, prev = n - 1, next = 0;
  bool failed = false;
  while (num > 3) {
    int found = 0;
    for (ear = next;; prev = ear, ear = next) {
      for (next = ear + 1; done[(next >= n ? next = 0 : next)]; ++next) {
      }
      if (next < ear && ++found == 2) break;
      const P2 &p1 = tv[ear], &p0 = tv[prev], &p2 = tv[next];
      if (on_left(p0, p2, p1)) continue;
      int k = 0;
      for (; k < n; ++k) {
        const P2& q = tv[k];
        const bool same1 = q.x == p1.x && q.y == p1.y, same2 = q.x == p2.x && q.y == p2.y,
                   same0 = q.x == p0.x && q.y == p0.y;
        if (!same1 && !same2 && !same0 && in_tri(p0, p1, p2, q)) break;
      }
      if (k != n) continue;
      break;
    }
    if (found == 2) {  // no ear: assimp gives up on the rest of the polygon
      failed = true;
      num = 0;
      break;
    }
    tri.insert(tri.end(), {prev, ear, next});
    done[ear] = 1;
    --num;
  }
  if (!failed && num > 0) {
    int k = 0;
    while (done[k]) ++k;
    const int a = k++;
    while (done[k]) ++k;
    const int b = k++;
    while (done[k]) ++k;
    tri.insert(tri.end(), {a, b, k});
  }
  for (size_t k = 0; k < tri.size(); k += 3) {  // drop 0-area triangles (projected area < 1e-5)
    if (std::fabs(area2d(tv[tri[k]], tv[tri[k + 1]], tv[tri[k + 2]])) < 1e-5f) continue;
    out.insert(out.end(), {base + (unsigned)tri[k], base + (unsigned)tri[k + 1], base + (unsigned)tri[k + 2]});
  }
}

std::string dir_of(const std::string& p) {
  const size_t s = p.find_last_of('/');
  return s == std::string::npos ? std::string() : p.substr(0, s + 1);
}

// Material library in definition order after assimp's default material (index 0), with each
// material's map_Kd (the file name is the last token of the line).
void read_mtl(const std::string& path, std::vector<std::string>& names, std::vector<std::string>& kd) {
  std::ifstream f(path);
  std::string line;
  int cur = -1;
  while (std::getline(f, line)) {
    std::istringstream ss(line);
    std::string tok;
    if (!(ss >> tok)) continue;
    if (tok == "newmtl") {
      std::string name;
      ss >> name;
      cur = -1;
      for (size_t k = 0; k < names.size(); ++k)
        if (names[k] == name) cur = (int)k;
      if (cur < 0) {
        names.push_back(name);
        kd.emplace_back();
        cur = (int)names.size() - 1;
      }
    } else if (tok == "map_Kd" && cur >= 0) {
      std::string last, t;
      while (ss >> t) last = t;
      kd[cur] = last;
    }
  }
}

// Parses corner "v", "v/t", "v//n", "v/t/n" (1-based or negative relative indices).
Corner parse_corner(const std::string& s, int nv, int nt, int nn) {
  Corner c{-1, -1, -1};
  int field = 0;
  size_t i = 0;
  while (i <= s.size()) {
    size_t j = s.find('/', i);
    if (j == std::string::npos) j = s.size();
    if (j > i) {
      const int v = std::atoi(s.substr(i, j - i).c_str());
      const int cnt = field == 0 ? nv : (field == 1 ? nt : nn);
      const int idx = v > 0 ? v - 1 : cnt + v;
      if (field == 0) c.v = idx; else if (field == 1) c.t = idx; else c.n = idx;
    }
    ++field;
    i = j + 1;
  }
  return c;
}

}  // namespace

struct rt_obj_mesh {
  rt_obj_info info{};
  std::vector<float> tris;
  std::string texture;
};

extern "C" {

int rt_obj_load(const char* path, int32_t index_mode, rt_obj_mesh** out) {
  if (!path || !out || (index_mode != RT_OBJ_INDEX_REFERENCE && index_mode != RT_OBJ_INDEX_GLOBAL)) return RT_ERR_ARG;
  *out = nullptr;
  std::ifstream f(path);
  if (!f) return RT_ERR_ARG;
  std::vector<P3> V, VN;
  std::vector<P2> VT;
  // ObjFileParser state (assimp): objects, meshes, current object / mesh / material.
  std::vector<Object> objs;
  std::vector<Mesh> meshes;
  std::vector<std::string> mat_names{"DefaultMaterial"}, kd{std::string()};
  int cur_obj = -1, cur_mesh = -1, cur_mat = -1;
  std::string active_group;
  auto create_mesh = [&]() {
    meshes.push_back(Mesh{});
    cur_mesh = (int)meshes.size() - 1;
    if (cur_obj >= 0) objs[cur_obj].meshes.push_back(cur_mesh);
  };
  auto create_object = [&](const std::string& name) {
    objs.push_back(Object{name, {}});
    cur_obj = (int)objs.size() - 1;
    create_mesh();
    if (cur_mat >= 0) meshes[cur_mesh].material = cur_mat;
  };
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream ss(line);
    std::string tok;
    if (!(ss >> tok)) continue;
    if (tok == "v" || tok == "vn") {
      std::string a, b, c;
      ss >> a >> b >> c;
      (tok == "v" ? V : VN).push_back(P3{atof_assimp(a.c_str()), atof_assimp(b.c_str()), atof_assimp(c.c_str())});
    } else if (tok == "vt") {
      std::string a, b;
      ss >> a >> b;
      VT.push_back(P2{atof_assimp(a.c_str()), b.empty() ? 0.0f : atof_assimp(b.c_str())});
    } else if (tok == "o") {  // getObjectName: re-activate an object of that name, else create one
      std::string name;
      std::getline(ss >> std::ws, name);
      int found = -1;
      for (size_t k = 0; k < objs.size(); ++k)
        if (objs[k].name == name) found = (int)k;
      if (found >= 0) cur_obj = found;
      else create_object(name);
    } else if (tok == "g") {  // getGroupName: a new group name maps to a new object
      std::string name;
      std::getline(ss >> std::ws, name);
      if (name != active_group) {
        create_object(name);
        active_group = name;
      }
    } else if (tok == "usemtl") {  // getMaterialDesc + needsNewMesh
      std::string name;
      ss >> name;
      if (cur_mat >= 0 && mat_names[cur_mat] == name) continue;
      int idx = 0;  // unknown names use the default material
      for (size_t k = 0; k < mat_names.size(); ++k)
        if (mat_names[k] == name) idx = (int)k;
      cur_mat = idx;
      const bool fresh = cur_mesh < 0 || (meshes[cur_mesh].material != kNoMaterial &&
                                           meshes[cur_mesh].material != idx && !meshes[cur_mesh].faces.empty());
      if (fresh) create_mesh();
      meshes[cur_mesh].material = idx;
    } else if (tok == "mtllib") {
      std::string name;
      ss >> name;
      read_mtl(dir_of(path) + name, mat_names, kd);
    } else if (tok == "f") {
      std::vector<Corner> face;
      std::string c;
      while (ss >> c) face.push_back(parse_corner(c, (int)V.size(), (int)VT.size(), (int)VN.size()));
      if (face.empty()) continue;
      if (cur_obj < 0) create_object("defaultobject");
      if (cur_mesh < 0) create_mesh();
      meshes[cur_mesh].faces.push_back(face);
    }
  }
  // processNode order: root has no meshes; children = objects in order, meshes in order.
  std::vector<P3> allv, alln;
  std::vector<P2> alluv;
  std::vector<unsigned> allidx;
  std::vector<unsigned> mesh_first_vertex;
  std::vector<std::string> tex_paths;
  std::unique_ptr<rt_obj_mesh> m(new rt_obj_mesh);
  for (const Object& o : objs) {
    for (int mi : o.meshes) {
      const Mesh& me = meshes[mi];
      if (me.faces.empty()) continue;
      std::vector<P3> mv, mn;
      std::vector<P2> muv;
      std::vector<unsigned> idx;
      // A mesh has normals when any corner has one (no GenNormals then); corners without a
      // normal or texture coordinate get zeros (createVertexArray).
      bool has_n = false;
      for (const auto& fc : me.faces)
        for (const Corner& c : fc) has_n = has_n || c.n >= 0;
      for (const auto& fc : me.faces) {
        const unsigned base = (unsigned)mv.size();
        std::vector<P3> pos;
        for (const Corner& c : fc) {
          const P3 p = c.v >= 0 && c.v < (int)V.size() ? V[c.v] : P3{0, 0, 0};
          mv.push_back(p);
          pos.push_back(p);
          mn.push_back(c.n >= 0 && c.n < (int)VN.size() ? VN[c.n] : P3{0, 0, 0});
          muv.push_back(c.t >= 0 && c.t < (int)VT.size() ? VT[c.t] : P2{0, 0});
        }
        if (fc.size() <= 3) {
          for (unsigned q = 0; q < fc.size(); ++q) idx.push_back(base + q);
        } else {
          triangulate(pos, base, idx);
        }
      }
      if (!has_n) {  // GenNormals -> per-face normals, later faces overwrite shared corners
        for (size_t k = 0; k + 2 < idx.size(); k += 3) {
          const P3 &a = mv[idx[k]], &b = mv[idx[k + 1]], &c = mv[idx[k + 2]];
          const P3 e1{b.x - a.x, b.y - a.y, b.z - a.z}, e2{c.x - a.x, c.y - a.y, c.z - a.z};
          P3 nrm{e1.y * e2.z - e1.z * e2.y, e1.z * e2.x - e1.x * e2.z, e1.x * e2.y - e1.y * e2.x};
          const float len = std::sqrt(nrm.x * nrm.x + nrm.y * nrm.y + nrm.z * nrm.z);
          if (len > 0.0f) nrm = P3{nrm.x / len, nrm.y / len, nrm.z / len};  // NormalizeSafe
          for (int q = 0; q < 3; ++q) mn[idx[k + q]] = nrm;
        }
      }
      if (me.material >= 0 && !kd[me.material].empty()) {  // processMesh: unique diffuse textures
        bool seen = false;
        for (const auto& t : tex_paths) seen = seen || t == kd[me.material];
        if (!seen) tex_paths.push_back(kd[me.material]);
      }
      mesh_first_vertex.push_back((unsigned)allv.size());
      const unsigned off = index_mode == RT_OBJ_INDEX_GLOBAL ? (unsigned)allv.size() : 0u;
      for (unsigned i : idx) allidx.push_back(i + off);
      allv.insert(allv.end(), mv.begin(), mv.end());
      alln.insert(alln.end(), mn.begin(), mn.end());
      alluv.insert(alluv.end(), muv.begin(), muv.end());
      ++m->info.n_meshes;
    }
  }
  // create_meshes_d: triangle j takes corners indices[3j..3j+2] of the concatenated arrays.
  const size_t nt = allidx.size() / 3;
  m->tris.resize(nt * 24);
  for (size_t j = 0; j < nt; ++j) {
    float* d = &m->tris[24 * j];
    for (int q = 0; q < 3; ++q) {
      const unsigned i = allidx[3 * j + q];
      if (i >= allv.size()) return RT_ERR_SCENE;
      d[3 * q + 0] = allv[i].x;
      d[3 * q + 1] = allv[i].y;
      d[3 * q + 2] = allv[i].z;
      d[9 + 3 * q + 0] = alln[i].x;
      d[9 + 3 * q + 1] = alln[i].y;
      d[9 + 3 * q + 2] = alln[i].z;
      d[18 + 2 * q + 0] = alluv[i].x;
      d[18 + 2 * q + 1] = alluv[i].y;
    }
  }
  m->texture = tex_paths.empty() ? std::string() : dir_of(path) + tex_paths[0];
  m->info.n_triangles = (int32_t)nt;
  m->info.n_textures = (int32_t)tex_paths.size();
  m->info.n_vertices = (int32_t)allv.size();
  m->info.triangles = m->tris.data();
  m->info.texture = m->texture.c_str();
  *out = m.release();
  return RT_OK;
}

const rt_obj_info* rt_obj_view(const rt_obj_mesh* m) { return m ? &m->info : nullptr; }

void rt_obj_free(rt_obj_mesh* m) { delete m; }

}  // extern "C"
