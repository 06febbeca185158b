// tree_lab — offline experiment: box/primitive tests per ray for traversal-tree designs over a
// captured ray set (oracle ref_capture_rays).  Not part of the product; design evidence only.
// build: g++ -O2 -std=c++17 scripts/tree_lab.cpp -Iinclude -Lraytracing_gpu_amd -lrt_hip \
//          -Wl,-rpath,$PWD/raytracing_gpu_amd -o /tmp/tree_lab
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#include "rt_hip.h"

struct Box {
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) lo[k] = std::min(lo[k], b.lo[k]), hi[k] = std::max(hi[k], b.hi[k]);
  }
  float area() const {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return dx < 0 ? 0 : 2 * (dx * dy + dy * dz + dz * dx);
  }
};
struct Ray {
  float o[3], d[3], tm, inv[3];
};

static const rt_prim* P;
static std::vector<Box> pbox;

static bool prim_hit(int pi, const Ray& r, float& t) {
  const rt_prim& q = P[pi];
  float c[3] = {q.p[0], q.p[1], q.p[2]};
  if (q.type == RT_PRIM_MOVING_SPHERE)
    for (int k = 0; k < 3; ++k) c[k] += ((r.tm - q.p[7]) / q.p[8]) * q.p[4 + k];
  float oc[3];
  for (int k = 0; k < 3; ++k) oc[k] = r.o[k] - c[k];
  const float a = r.d[0] * r.d[0] + r.d[1] * r.d[1] + r.d[2] * r.d[2];
  const float hb = oc[0] * r.d[0] + oc[1] * r.d[1] + oc[2] * r.d[2];
  const float cc = oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2] - q.p[3] * q.p[3];
  const float disc = hb * hb - a * cc;
  if (disc < 0) return false;
  const float root = (-hb - std::sqrt(disc)) / a;
  if (root < 0.001f) return false;
  t = root;
  return true;
}
static bool box_hit(const Box& b, const Ray& r, float tmax, float& tn) {
  float t0 = 0.001f, t1 = tmax;
  for (int k = 0; k < 3; ++k) {
    float a = (b.lo[k] - r.o[k]) * r.inv[k], c = (b.hi[k] - r.o[k]) * r.inv[k];
    if (a > c) std::swap(a, c);
    if (a == a) t0 = std::max(t0, a);
    if (c == c) t1 = std::min(t1, c);
  }
  tn = t0;
  return t0 <= t1;
}

// Generic binary tree: node children (>=0 inner, <0 leaf -> prim list), child boxes in parent.
struct Node {
  Box cb[2];
  int child[2];
};
struct Tree {
  std::vector<Node> nodes;
  std::vector<std::vector<int>> leaves;  // leaf id -> prims
  Box root_box;
};

static int build_sah(Tree& T, std::vector<int> ids, int maxleaf, int depth, int& maxdepth) {
  maxdepth = std::max(maxdepth, depth);
  Box b;
  for (int id : ids) b.grow(pbox[id]);
  if ((int)ids.size() <= maxleaf) {
    T.leaves.push_back(ids);
    return -(int)T.leaves.size();
  }
  float best = INFINITY;
  int bax = -1, bsplit = -1;
  for (int ax = 0; ax < 3; ++ax) {
    std::sort(ids.begin(), ids.end(), [&](int x, int y) {
      return pbox[x].lo[ax] + pbox[x].hi[ax] < pbox[y].lo[ax] + pbox[y].hi[ax];
    });
    const int n = (int)ids.size();
    std::vector<float> right(n + 1, 0);
    Box acc;
    for (int i = n - 1; i >= 1; --i) {
      acc.grow(pbox[ids[i]]);
      right[i] = acc.area() * (n - i);
    }
    Box lacc;
    for (int i = 1; i < n; ++i) {
      lacc.grow(pbox[ids[i - 1]]);
      const float cost = lacc.area() * i + right[i];
      if (cost < best) best = cost, bax = ax, bsplit = i;
    }
  }
  std::sort(ids.begin(), ids.end(), [&](int x, int y) {
    return pbox[x].lo[bax] + pbox[x].hi[bax] < pbox[y].lo[bax] + pbox[y].hi[bax];
  });
  std::vector<int> L(ids.begin(), ids.begin() + bsplit), R(ids.begin() + bsplit, ids.end());
  const int me = (int)T.nodes.size();
  T.nodes.push_back(Node{});
  Box lb, rb;
  for (int id : L) lb.grow(pbox[id]);
  for (int id : R) rb.grow(pbox[id]);
  const int cl = build_sah(T, L, maxleaf, depth + 1, maxdepth);
  const int cr = build_sah(T, R, maxleaf, depth + 1, maxdepth);
  T.nodes[me].cb[0] = lb;
  T.nodes[me].cb[1] = rb;
  T.nodes[me].child[0] = cl;
  T.nodes[me].child[1] = cr;
  return me;
}

// Median perfect tree (the current traversal tree): leaves of 1-2 prims, largest-extent splits.
static int build_median(Tree& T, std::vector<int> ids, const std::vector<int>& num, int k, int last0) {
  if (k >= last0) {
    T.leaves.push_back(ids);
    return -(int)T.leaves.size();
  }
  Box c;
  for (int id : ids)
    for (int a = 0; a < 3; ++a) {
      const float m = 0.5f * pbox[id].lo[a] + 0.5f * pbox[id].hi[a];
      c.lo[a] = std::min(c.lo[a], m), c.hi[a] = std::max(c.hi[a], m);
    }
  int ax = 0;
  for (int a = 1; a < 3; ++a)
    if (c.hi[a] - c.lo[a] > c.hi[ax] - c.lo[ax]) ax = a;
  std::stable_sort(ids.begin(), ids.end(), [&](int x, int y) {
    return 0.5f * pbox[x].lo[ax] + 0.5f * pbox[x].hi[ax] < 0.5f * pbox[y].lo[ax] + 0.5f * pbox[y].hi[ax];
  });
  const int nl = num[2 * k + 1];
  std::vector<int> L(ids.begin(), ids.begin() + nl), R(ids.begin() + nl, ids.end());
  const int me = (int)T.nodes.size();
  T.nodes.push_back(Node{});
  Box lb, rb;
  for (int id : L) lb.grow(pbox[id]);
  for (int id : R) rb.grow(pbox[id]);
  const int cl = build_median(T, L, num, 2 * k + 1, last0);
  const int cr = build_median(T, R, num, 2 * k + 2, last0);
  T.nodes[me].cb[0] = lb;
  T.nodes[me].cb[1] = rb;
  T.nodes[me].child[0] = cl;
  T.nodes[me].child[1] = cr;
  return me;
}

struct Stats {
  double box = 0, prim = 0, steps = 0, maxstack = 0;
};
static void trace(const Tree& T, const Ray& r, Stats& st) {
  float best = INFINITY;
  int stack[64], sp = 0;
  int cur = 0;
  for (;;) {
    if (cur < 0) {
      for (int id : T.leaves[-cur - 1]) {
        float t;
        st.prim++;
        if (prim_hit(id, r, t) && t < best) best = t;
      }
    } else {
      st.steps++;
      const Node& n = T.nodes[cur];
      float t0, t1;
      const float cut = best * 1.0039f;
      st.box += 2;
      const bool h0 = box_hit(n.cb[0], r, cut, t0), h1 = box_hit(n.cb[1], r, cut, t1);
      if (h0 && h1) {
        const bool f = t1 < t0;
        stack[sp++] = n.child[f ? 0 : 1];
        st.maxstack = std::max(st.maxstack, (double)sp);
        cur = n.child[f ? 1 : 0];
        continue;
      }
      if (h0 || h1) {
        cur = n.child[h0 ? 0 : 1];
        continue;
      }
    }
    if (sp == 0) break;
    cur = stack[--sp];
  }
}

// Device scheme: leaf size 1, prim children tested inside the parent's step.
static void trace_inline(const Tree& T, const Ray& r, Stats& st) {
  float best = INFINITY;
  int stack[64], sp = 0;
  int cur = 0;
  for (;;) {
    st.steps++;
    const Node& n = T.nodes[cur];
    float tt[2];
    const float cut = best * 1.0039f;
    st.box += 2;
    bool h[2] = {box_hit(n.cb[0], r, cut, tt[0]), box_hit(n.cb[1], r, cut, tt[1])};
    for (int c = 0; c < 2; ++c)
      if (h[c] && n.child[c] < 0) {
        float t;
        st.prim++;
        for (int id : T.leaves[-n.child[c] - 1])
          if (prim_hit(id, r, t) && t < best) best = t;
        h[c] = false;
      }
    if (h[0] && h[1]) {
      const bool f = tt[1] < tt[0];
      stack[sp++] = n.child[f ? 0 : 1];
      st.maxstack = std::max(st.maxstack, (double)sp);
      cur = n.child[f ? 1 : 0];
      continue;
    }
    if (h[0] || h[1]) {
      cur = n.child[h[0] ? 0 : 1];
      continue;
    }
    if (sp == 0) break;
    cur = stack[--sp];
  }
}


// 4-wide collapse of a binary tree: each node takes its children, replacing inner children by
// their two children (2..4 children per node); leaves stay leaves (one primitive each).
struct Node4 {
  Box cb[4];
  int child[4];  // >= 0: Node4 index, < 0: leaf
  int n = 0;
};
static int collapse4(const Tree& T, int k, std::vector<Node4>& out) {
  const int me = (int)out.size();
  out.push_back(Node4{});
  Node4 m;
  const Node& b = T.nodes[k];
  std::vector<std::pair<Box, int>> kids;
  for (int c = 0; c < 2; ++c) {
    if (b.child[c] < 0) {
      kids.push_back({b.cb[c], b.child[c]});
    } else {
      const Node& g = T.nodes[b.child[c]];
      for (int d = 0; d < 2; ++d) kids.push_back({g.cb[d], g.child[d]});
    }
  }
  for (auto& kd : kids) {
    m.cb[m.n] = kd.first;
    m.child[m.n] = kd.second;  // binary index for now
    ++m.n;
  }
  for (int c = 0; c < m.n; ++c)
    if (m.child[c] >= 0) m.child[c] = collapse4(T, m.child[c], out);
  out[me] = m;
  return me;
}
static void trace4(const Tree& T, const std::vector<Node4>& N, const Ray& r, Stats& st) {
  float best = INFINITY;
  int stack[128], sp = 0;
  int cur = 0;
  for (;;) {
    st.steps++;
    const Node4& n = N[cur];
    const float cut = best * 1.0039f;
    float tt[4];
    int hit_inner[4], ni = 0;
    for (int c = 0; c < n.n; ++c) {
      st.box += 1;
      if (!box_hit(n.cb[c], r, cut, tt[c])) continue;
      if (n.child[c] < 0) {
        float t;
        st.prim++;
        for (int id : T.leaves[-n.child[c] - 1])
          if (prim_hit(id, r, t) && t < best) best = t;
      } else {
        hit_inner[ni++] = c;
      }
    }
    // nearest first: push the others far-to-near
    std::sort(hit_inner, hit_inner + ni, [&](int a, int b) { return tt[a] > tt[b]; });
    for (int q = 0; q + 1 < ni; ++q) stack[sp++] = n.child[hit_inner[q]];
    st.maxstack = std::max(st.maxstack, (double)sp);
    if (ni > 0) {
      cur = n.child[hit_inner[ni - 1]];
      continue;
    }
    if (sp == 0) break;
    cur = stack[--sp];
  }
}

int main(int argc, char** argv) {
  const char* rays_path = argc > 1 ? argv[1] : "/tmp/c2_rays.bin";
  FILE* f = fopen(rays_path, "rb");
  std::vector<float> raw;
  float buf[8];
  while (fread(buf, 4, 8, f) == 8) raw.insert(raw.end(), buf, buf + 8);
  fclose(f);
  const size_t nr = raw.size() / 8;
  std::vector<Ray> rays(nr);
  for (size_t i = 0; i < nr; ++i) {
    Ray& r = rays[i];
    for (int k = 0; k < 3; ++k) r.o[k] = raw[8 * i + k], r.d[k] = raw[8 * i + 3 + k], r.inv[k] = 1.0f / r.d[k];
    r.tm = raw[8 * i + 6];
  }
  rt_scene_host* sh;
  rt_scene_build("big1", &sh);
  const rt_scene_soa* s = rt_scene_view(sh);
  P = s->prims;
  const int n = s->n_prims;
  pbox.resize(n);
  for (int i = 0; i < n; ++i) {
    const rt_prim& q = P[i];
    Box b;
    float c0[3] = {q.p[0], q.p[1], q.p[2]}, c1[3] = {q.p[0], q.p[1], q.p[2]};
    if (q.type == RT_PRIM_MOVING_SPHERE)
      for (int k = 0; k < 3; ++k) c1[k] += q.p[4 + k];
    for (int k = 0; k < 3; ++k) {
      b.lo[k] = std::min(c0[k], c1[k]) - q.p[3];
      b.hi[k] = std::max(c0[k], c1[k]) + q.p[3];
    }
    pbox[i] = b;
  }
  std::vector<int> all(n);
  for (int i = 0; i < n; ++i) all[i] = i;
  auto run = [&](const char* name, Tree& T, int depth) {
    Stats st;
    for (const Ray& r : rays) trace(T, r, st);
    printf("%-18s nodes %4zu depth %2d | per ray: box %6.2f prim %5.2f steps %5.2f maxstack %2.0f\n", name,
           T.nodes.size(), depth, st.box / nr, st.prim / nr, st.steps / nr, st.maxstack);
  };
  {
    int rows = 0;
    while ((1 << rows) < n) ++rows;
    const int inner = (1 << rows) - 1, last0 = (1 << (rows - 1)) - 1;
    std::vector<int> num(inner);
    num[0] = n;
    for (int k = 1; k < inner; ++k) num[k] = (k & 1) ? num[(k - 1) / 2] / 2 : num[(k - 1) / 2] / 2 + num[(k - 1) / 2] % 2;
    Tree T;
    build_median(T, all, num, 0, last0);
    run("median-perfect", T, rows);
  }
  for (int leaf : {1, 2, 3, 4}) {
    Tree T;
    int md = 0;
    build_sah(T, all, leaf, 0, md);
    char nm[32];
    snprintf(nm, sizeof nm, "sah-leaf%d", leaf);
    run(nm, T, md);
    if (leaf == 1) {
      Stats st;
      std::vector<int> hist(256, 0);
      double wave_max = 0, wave_sum = 0;
      int lane = 0, cur_max = 0;
      for (const Ray& r : rays) {
        Stats one;
        trace_inline(T, r, one);
        st.box += one.box; st.prim += one.prim; st.steps += one.steps; st.maxstack = std::max(st.maxstack, one.maxstack);
        hist[std::min(255, (int)one.steps)]++;
        cur_max = std::max(cur_max, (int)one.steps);
        if (++lane == 64) { wave_max += cur_max; wave_sum += 1; lane = 0; cur_max = 0; }
      }
      long long acc = 0; int p50=0,p90=0,p99=0;
      for (int i = 0; i < 256; ++i) { acc += hist[i]; if (!p50 && acc >= 0.5*nr) p50=i; if (!p90 && acc >= 0.9*nr) p90=i; if (!p99 && acc >= 0.99*nr) p99=i; }
      printf("steps p50 %d p90 %d p99 %d; mean over consecutive 64-ray groups of max steps: %.1f\n", p50, p90, p99, wave_max / wave_sum);
      printf("%-18s nodes %4zu depth %2d | per ray: box %6.2f prim %5.2f steps %5.2f maxstack %2.0f\n",
             "sah1-inline-prims", T.nodes.size(), md, st.box / nr, st.prim / nr, st.steps / nr, st.maxstack);
      std::vector<Node4> N4;
      collapse4(T, 0, N4);
      Stats s4;
      double wmax = 0, wsum = 0;
      int ln = 0, cm = 0;
      for (const Ray& r : rays) {
        Stats one;
        trace4(T, N4, r, one);
        s4.box += one.box; s4.prim += one.prim; s4.steps += one.steps; s4.maxstack = std::max(s4.maxstack, one.maxstack);
        cm = std::max(cm, (int)one.steps);
        if (++ln == 64) { wmax += cm; wsum += 1; ln = 0; cm = 0; }
      }
      printf("%-18s nodes %4zu        | per ray: box %6.2f prim %5.2f steps %5.2f maxstack %2.0f wave-max steps %.1f\n",
             "sah1-bvh4", N4.size(), s4.box / nr, s4.prim / nr, s4.steps / nr, s4.maxstack, wmax / wsum);
    }
  }
  printf("rays %zu\n", nr);
  return 0;
}
