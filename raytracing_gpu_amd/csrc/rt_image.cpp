// rt_image.cpp — baseline JPEG decoding for scene textures: the host side of make_image() /
// imread() (texture.h:166-203), which the reference runs through its vendored stb_image v2.26
// (stbi_load(path, &w, &h, &n, 0)).
//
// The texels a texture lookup returns are the decoder's output bytes, so this file restates the
// arithmetic stb_image uses for baseline (sequential Huffman) JPEGs, where decoders differ:
//   * the integer IDCT derived from libjpeg's jidctint (12-bit fixed-point constants rounded
//     from float, 2 extra bits between passes, a DC-only column shortcut, +128 and clamp);
//   * component planes padded to whole MCUs;
//   * chroma upsampling: none, 2x horizontal / vertical (3:1 triangle, +2 >> 2), or 2x2
//     (3:1 in both directions, +8 >> 4 between samples, +2 >> 2 at the row ends), with the
//     near/far source rows chosen per output row as stb's resampler steps through them;
//   * YCbCr -> RGB in 20-bit fixed point with constants rounded from float and the G term's Cb
//     product truncated to its upper 16 bits.
// Pinned bit-exact against the reference's own stb_image (compiled in place under oracle/_ref
// by `make -C oracle ref`) on the reference's textures (tests/test_image_cpu.py).
// Progressive and arithmetic-coded JPEGs are rejected (neither occurs in the reference's assets).
#include <algorithm>
#include <cstdint>
#include <iterator>
#include <string>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <vector>

#include "../../include/rt_hip.h"

namespace {

const uint8_t kDezigzag[64 + 15] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
                                    // guard entries for corrupt run lengths
                                    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct Huff {
  // canonical code tables: for each code length L, codes [mincode[L], maxcode[L]] map to
  // values starting at valptr[L]
  int mincode[17] = {}, maxcode[18] = {}, valptr[17] = {};
  uint8_t vals[256] = {};
  bool present = false;  // defined by a DHT segment
};

struct Comp {
  int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
  int x = 0, y = 0, w2 = 0, h2 = 0;  // valid size, padded plane size
  int dc_pred = 0;
  std::vector<uint8_t> plane;
};

struct Jpeg {
  const uint8_t* p;
  const uint8_t* end;
  uint16_t dequant[4][64] = {};
  Huff dc[4], ac[4];
  Comp comp[4];
  int ncomp = 0, width = 0, height = 0, hmax = 1, vmax = 1, restart = 0;
  bool jfif = false, adobe_rgb = false;
  int app14_transform = -1;
  // bit reader
  uint32_t bitbuf = 0;
  int bitcnt = 0;
  bool hit_marker = false;
  std::string err;

  int byte() { return p < end ? *p++ : 0; }
  int be16() {
    const int a = byte();
    return (a << 8) | byte();
  }
  void fill() {
    while (bitcnt <= 24) {
      int b = 0;
      if (!hit_marker) {
        b = byte();
        if (b == 0xff) {
          int c = byte();
          while (c == 0xff) c = byte();
          if (c != 0) {  // a marker: feed zeros from here on
            hit_marker = true;
            p -= 2;
            b = 0;
          }
        }
      }
      bitbuf |= (uint32_t)b << (24 - bitcnt);
      bitcnt += 8;
    }
  }
  int bits(int n) {  // n <= 16
    if (n == 0) return 0;
    if (bitcnt < n) fill();
    const int v = (int)(bitbuf >> (32 - n));
    bitbuf <<= n;
    bitcnt -= n;
    return v;
  }
  int bit() { return bits(1); }
  int decode(const Huff& h) {
    int code = 0;
    for (int l = 1; l <= 16; ++l) {
      code = (code << 1) | bit();
      if (h.maxcode[l] >= 0 && code <= h.maxcode[l] && code >= h.mincode[l]) return h.vals[h.valptr[l] + code - h.mincode[l]];
    }
    return -1;
  }
  // EXTEND of the JPEG spec: an s-bit magnitude category to a signed value.
  int receive_extend(int s) {
    if (s == 0) return 0;
    const int v = bits(s);
    return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v;
  }
  void reset_bits() {
    bitbuf = 0;
    bitcnt = 0;
    hit_marker = false;
  }
};

inline uint8_t clamp255(int x) { return x < 0 ? 0 : (x > 255 ? 255 : (uint8_t)x); }

// 12-bit fixed-point IDCT constants, rounded from float: (int)(c * 4096 + 0.5).
constexpr int fx(float c) { return (int)((double)(c * 4096.0f) + 0.5); }

// Attribution: idct_1d / idct_block follow stb_image v2.26's stbi__idct_block (Sean Barrett,
// public domain / MIT; vendored by the reference at external/stb_image.h:2356-2449), itself
// derived from the IJG's jidctint.c: bit-exact texels need the identical integer arithmetic.
// One 1-D pass of the jidctint-derived IDCT over s0..s7; outputs the even part x0..x3 and
// odd part t0..t3 (results are x_k +- t_(3-k)).
inline void idct_1d(int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7, int& x0, int& x1, int& x2,
                    int& x3, int& t0, int& t1, int& t2, int& t3) {
  int p1, p2, p3, p4, p5;
  p2 = s2;
  p3 = s6;
  p1 = (p2 + p3) * fx(0.5411961f);
  t2 = p1 + p3 * fx(-1.847759065f);
  t3 = p1 + p2 * fx(0.765366865f);
  p2 = s0;
  p3 = s4;
  t0 = (p2 + p3) * 4096;
  t1 = (p2 - p3) * 4096;
  x0 = t0 + t3;
  x3 = t0 - t3;
  x1 = t1 + t2;
  x2 = t1 - t2;
  t0 = s7;
  t1 = s5;
  t2 = s3;
  t3 = s1;
  p3 = t0 + t2;
  p4 = t1 + t3;
  p1 = t0 + t3;
  p2 = t1 + t2;
  p5 = (p3 + p4) * fx(1.175875602f);
  t0 = t0 * fx(0.298631336f);
  t1 = t1 * fx(2.053119869f);
  t2 = t2 * fx(3.072711026f);
  t3 = t3 * fx(1.501321110f);
  p1 = p5 + p1 * fx(-0.899976223f);
  p2 = p5 + p2 * fx(-2.562915447f);
  p3 = p3 * fx(-1.961570560f);
  p4 = p4 * fx(-0.390180644f);
  t3 += p1 + p4;
  t2 += p2 + p3;
  t1 += p2 + p4;
  t0 += p1 + p3;
}

void idct_block(uint8_t* out, int stride, const short* d) {
  int val[64];
  for (int c = 0; c < 8; ++c) {  // columns, 2 extra bits kept
    const short* s = d + c;
    int* v = val + c;
    if (s[8] == 0 && s[16] == 0 && s[24] == 0 && s[32] == 0 && s[40] == 0 && s[48] == 0 && s[56] == 0) {
      const int dc = s[0] * 4;
      for (int r = 0; r < 8; ++r) v[8 * r] = dc;
      continue;
    }
    int x0, x1, x2, x3, t0, t1, t2, t3;
    idct_1d(s[0], s[8], s[16], s[24], s[32], s[40], s[48], s[56], x0, x1, x2, x3, t0, t1, t2, t3);
    x0 += 512;
    x1 += 512;
    x2 += 512;
    x3 += 512;
    v[0] = (x0 + t3) >> 10;
    v[56] = (x0 - t3) >> 10;
    v[8] = (x1 + t2) >> 10;
    v[48] = (x1 - t2) >> 10;
    v[16] = (x2 + t1) >> 10;
    v[40] = (x2 - t1) >> 10;
    v[24] = (x3 + t0) >> 10;
    v[32] = (x3 - t0) >> 10;
  }
  for (int r = 0; r < 8; ++r) {  // rows: remove 1<<17 with rounding, +128 level shift
    const int* v = val + 8 * r;
    uint8_t* o = out + r * stride;
    int x0, x1, x2, x3, t0, t1, t2, t3;
    idct_1d(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], x0, x1, x2, x3, t0, t1, t2, t3);
    const int bias = 65536 + (128 << 17);
    x0 += bias;
    x1 += bias;
    x2 += bias;
    x3 += bias;
    o[0] = clamp255((x0 + t3) >> 17);
    o[7] = clamp255((x0 - t3) >> 17);
    o[1] = clamp255((x1 + t2) >> 17);
    o[6] = clamp255((x1 - t2) >> 17);
    o[2] = clamp255((x2 + t1) >> 17);
    o[5] = clamp255((x2 - t1) >> 17);
    o[3] = clamp255((x3 + t0) >> 17);
    o[4] = clamp255((x3 - t0) >> 17);
  }
}

bool build_huff(Huff& h, const uint8_t counts[16], const uint8_t* vals, int nvals) {
  int code = 0, k = 0;
  for (int l = 1; l <= 16; ++l) {
    h.valptr[l] = k;
    h.mincode[l] = code;
    code += counts[l - 1];
    k += counts[l - 1];
    h.maxcode[l] = counts[l - 1] ? code - 1 : -1;
    if (code > (1 << l)) return false;
    code <<= 1;
  }
  if (nvals > 256) return false;
  memcpy(h.vals, vals, (size_t)nvals);
  h.present = true;
  return true;
}

// One 8x8 block of a baseline scan: DC difference, AC run-lengths, dequantised in natural order.
bool decode_block(Jpeg& j, short data[64], Comp& c) {
  memset(data, 0, 64 * sizeof(short));
  const uint16_t* dq = j.dequant[c.tq];
  const int t = j.decode(j.dc[c.td]);
  if (t < 0 || t > 15) return false;
  const int dc = c.dc_pred + j.receive_extend(t);
  c.dc_pred = dc;
  data[0] = (short)(dc * dq[0]);
  int k = 1;
  while (k < 64) {
    const int rs = j.decode(j.ac[c.ta]);
    if (rs < 0) return false;
    const int s = rs & 15, r = rs >> 4;
    if (s == 0) {
      if (rs != 0xf0) break;  // end of block
      k += 16;
      continue;
    }
    k += r;
    const int zig = kDezigzag[k++];
    data[zig] = (short)(j.receive_extend(s) * dq[zig]);
  }
  return true;
}

bool read_restart(Jpeg& j) {
  j.reset_bits();
  // skip to the RSTn marker
  while (j.p + 1 < j.end && !(j.p[0] == 0xff && j.p[1] >= 0xd0 && j.p[1] <= 0xd7)) ++j.p;
  if (j.p + 1 >= j.end) return false;
  j.p += 2;
  for (int k = 0; k < j.ncomp; ++k) j.comp[k].dc_pred = 0;
  return true;
}

bool decode_scan(Jpeg& j, const int* scomp, int ns) {
  j.reset_bits();
  for (int k = 0; k < j.ncomp; ++k) j.comp[k].dc_pred = 0;
  short data[64];
  int todo = j.restart ? j.restart : 0x7fffffff;
  if (ns == 1) {  // non-interleaved: the component's own block grid
    Comp& c = j.comp[scomp[0]];
    const int bw = (c.x + 7) >> 3, bh = (c.y + 7) >> 3;
    for (int by = 0; by < bh; ++by)
      for (int bx = 0; bx < bw; ++bx) {
        if (!decode_block(j, data, c)) return false;
        idct_block(c.plane.data() + (size_t)c.w2 * by * 8 + bx * 8, c.w2, data);
        if (--todo <= 0 && !(by == bh - 1 && bx == bw - 1)) {
          if (!read_restart(j)) return false;
          todo = j.restart;
        }
      }
    return true;
  }
  const int mx = (j.width + 8 * j.hmax - 1) / (8 * j.hmax), my = (j.height + 8 * j.vmax - 1) / (8 * j.vmax);
  for (int y = 0; y < my; ++y)
    for (int x = 0; x < mx; ++x) {
      for (int q = 0; q < ns; ++q) {
        Comp& c = j.comp[scomp[q]];
        for (int v = 0; v < c.v; ++v)
          for (int h = 0; h < c.h; ++h) {
            if (!decode_block(j, data, c)) return false;
            const int bx = (x * c.h + h) * 8, byy = (y * c.v + v) * 8;
            idct_block(c.plane.data() + (size_t)c.w2 * byy + bx, c.w2, data);
          }
      }
      if (--todo <= 0 && !(y == my - 1 && x == mx - 1)) {
        if (!read_restart(j)) return false;
        todo = j.restart;
      }
    }
  return true;
}

bool parse(Jpeg& j) {
  if (j.byte() != 0xff || j.byte() != 0xd8) return (j.err = "not a JPEG", false);
  bool have_frame = false;
  for (;;) {
    int m = j.byte();
    while (m != 0xff && j.p < j.end) m = j.byte();  // resync
    if (j.p >= j.end) return (j.err = "truncated", false);
    int marker = j.byte();
    while (marker == 0xff) marker = j.byte();
    if (marker == 0xd9) break;                            // EOI
    if (marker == 0xd8 || (marker >= 0xd0 && marker <= 0xd7)) continue;
    const int len = j.be16();
    const uint8_t* seg_end = j.p + len - 2;
    if (len < 2 || seg_end > j.end) return (j.err = "bad segment", false);
    if (marker == 0xc0 || marker == 0xc1) {  // baseline / extended sequential Huffman
      if (j.byte() != 8) return (j.err = "only 8-bit JPEGs", false);
      j.height = j.be16();
      j.width = j.be16();
      j.ncomp = j.byte();
      if (j.ncomp != 1 && j.ncomp != 3) return (j.err = "only grey or 3-component JPEGs", false);
      for (int k = 0; k < j.ncomp; ++k) {
        Comp& c = j.comp[k];
        c.id = j.byte();
        const int hv = j.byte();
        c.h = hv >> 4;
        c.v = hv & 15;
        c.tq = j.byte() & 3;
        if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4) return (j.err = "bad sampling", false);
        j.hmax = std::max(j.hmax, c.h);
        j.vmax = std::max(j.vmax, c.v);
      }
      if (j.ncomp == 3 && j.comp[0].id == 'R' && j.comp[1].id == 'G' && j.comp[2].id == 'B') j.adobe_rgb = true;
      const int mx = (j.width + 8 * j.hmax - 1) / (8 * j.hmax), my = (j.height + 8 * j.vmax - 1) / (8 * j.vmax);
      for (int k = 0; k < j.ncomp; ++k) {
        Comp& c = j.comp[k];
        c.x = (j.width * c.h + j.hmax - 1) / j.hmax;
        c.y = (j.height * c.v + j.vmax - 1) / j.vmax;
        c.w2 = mx * c.h * 8;
        c.h2 = my * c.v * 8;
        c.plane.assign((size_t)c.w2 * c.h2, 0);
      }
      have_frame = true;
    } else if (marker >= 0xc2 && marker <= 0xcf && marker != 0xc4 && marker != 0xc8 && marker != 0xcc) {
      return (j.err = "progressive / lossless / arithmetic JPEGs are not supported", false);
    } else if (marker == 0xdb) {  // DQT
      while (j.p < seg_end) {
        const int pq = j.byte();
        const int t = pq & 15;
        const bool sixteen = (pq >> 4) != 0;
        if (t > 3) return (j.err = "bad DQT", false);
        for (int i = 0; i < 64; ++i) j.dequant[t][kDezigzag[i]] = (uint16_t)(sixteen ? j.be16() : j.byte());
      }
    } else if (marker == 0xc4) {  // DHT
      while (j.p < seg_end) {
        const int tc = j.byte();
        uint8_t counts[16];
        int n = 0;
        for (int i = 0; i < 16; ++i) n += (counts[i] = (uint8_t)j.byte());
        if (n > 256 || j.p + n > seg_end) return (j.err = "bad DHT", false);
        Huff& h = (tc >> 4) ? j.ac[tc & 3] : j.dc[tc & 3];
        if (!build_huff(h, counts, j.p, n)) return (j.err = "bad DHT", false);
        j.p += n;
      }
    } else if (marker == 0xdd) {  // DRI
      j.restart = j.be16();
    } else if (marker == 0xda) {  // SOS
      if (!have_frame) return (j.err = "scan before frame", false);
      const int ns = j.byte();
      int scomp[4];
      if (ns < 1 || ns > 4) return (j.err = "bad SOS", false);
      for (int q = 0; q < ns; ++q) {
        const int id = j.byte(), tt = j.byte();
        int k = 0;
        while (k < j.ncomp && j.comp[k].id != id) ++k;
        if (k == j.ncomp) return (j.err = "bad SOS component", false);
        // stb_image v2.26 rejects selectors past its 4 tables ('bad DC huff' / 'bad AC huff')
        if ((tt >> 4) > 3) return (j.err = "bad DC huff", false);
        if ((tt & 15) > 3) return (j.err = "bad AC huff", false);
        j.comp[k].td = tt >> 4;
        j.comp[k].ta = tt & 15;
        // a scan may only select tables a DHT segment defined
        if (!j.dc[j.comp[k].td].present || !j.ac[j.comp[k].ta].present)
          return (j.err = "scan selects an undefined Huffman table", false);
        scomp[q] = k;
      }
      j.p = seg_end;  // Ss, Se, Ah/Al: sequential baseline ignores them
      if (!decode_scan(j, scomp, ns)) return (j.err.empty() ? j.err = "corrupt scan" : j.err, false);
      // continue after the entropy-coded data: find the next marker
      while (j.p + 1 < j.end && !(j.p[0] == 0xff && j.p[1] != 0 && !(j.p[1] >= 0xd0 && j.p[1] <= 0xd7))) ++j.p;
      continue;
    } else {
      if (marker == 0xe0 && len >= 7 && !memcmp(j.p, "JFIF\0", 5)) j.jfif = true;
      if (marker == 0xee && len >= 14 && !memcmp(j.p, "Adobe", 5)) j.app14_transform = j.p[11];
    }
    j.p = seg_end;
  }
  return have_frame ? true : (j.err = "no frame", false);
}

// Row resamplers: out gets `2w` (or w) samples of one upsampled row from the near/far rows.
const uint8_t* row_1(uint8_t*, const uint8_t* near, const uint8_t*, int) { return near; }
const uint8_t* row_v2(uint8_t* out, const uint8_t* near, const uint8_t* far, int w) {
  for (int i = 0; i < w; ++i) out[i] = (uint8_t)((3 * near[i] + far[i] + 2) >> 2);
  return out;
}
const uint8_t* row_h2(uint8_t* out, const uint8_t* in, const uint8_t*, int w) {
  if (w == 1) {
    out[0] = out[1] = in[0];
    return out;
  }
  out[0] = in[0];
  out[1] = (uint8_t)((in[0] * 3 + in[1] + 2) >> 2);
  int i = 1;
  for (; i < w - 1; ++i) {
    const int n = 3 * in[i] + 2;
    out[2 * i] = (uint8_t)((n + in[i - 1]) >> 2);
    out[2 * i + 1] = (uint8_t)((n + in[i + 1]) >> 2);
  }
  out[2 * i] = (uint8_t)((in[w - 2] * 3 + in[w - 1] + 2) >> 2);
  out[2 * i + 1] = in[w - 1];
  return out;
}
const uint8_t* row_hv2(uint8_t* out, const uint8_t* near, const uint8_t* far, int w) {
  if (w == 1) {
    out[0] = out[1] = (uint8_t)((3 * near[0] + far[0] + 2) >> 2);
    return out;
  }
  int t1 = 3 * near[0] + far[0];
  out[0] = (uint8_t)((t1 + 2) >> 2);
  for (int i = 1; i < w; ++i) {
    const int t0 = t1;
    t1 = 3 * near[i] + far[i];
    out[2 * i - 1] = (uint8_t)((3 * t0 + t1 + 8) >> 4);
    out[2 * i] = (uint8_t)((3 * t1 + t0 + 8) >> 4);
  }
  out[2 * w - 1] = (uint8_t)((t1 + 2) >> 2);
  return out;
}
const uint8_t* row_generic(uint8_t* out, const uint8_t* near, const uint8_t*, int w, int hs) {
  for (int i = 0; i < w; ++i)
    for (int k = 0; k < hs; ++k) out[i * hs + k] = near[i];
  return out;
}

constexpr int fx20(float c) { return ((int)(c * 4096.0f + 0.5f)) << 8; }

void ycbcr_row(uint8_t* out, const uint8_t* y, const uint8_t* cb, const uint8_t* cr, int n, int step) {
  for (int i = 0; i < n; ++i) {
    const int yf = (y[i] << 20) + (1 << 19);
    const int vr = cr[i] - 128, vb = cb[i] - 128;
    int r = yf + vr * fx20(1.40200f);
    int g = yf + (vr * -fx20(0.71414f)) + ((vb * -fx20(0.34414f)) & (int)0xffff0000);
    int b = yf + vb * fx20(1.77200f);
    r >>= 20;
    g >>= 20;
    b >>= 20;
    out[0] = clamp255(r);
    out[1] = clamp255(g);
    out[2] = clamp255(b);
    out += step;
  }
}

}  // namespace

struct rt_image_host {
  rt_image_asset view{};
  std::vector<uint8_t> px;
  std::string err;
};

extern "C" {

int rt_image_decode(const uint8_t* bytes, int64_t n, rt_image_host** out) {
  if (!bytes || n <= 0 || !out) return RT_ERR_ARG;
  *out = nullptr;
  std::unique_ptr<Jpeg> j(new Jpeg());
  j->p = bytes;
  j->end = bytes + n;
  memset(j->dequant, 0, sizeof(j->dequant));
  if (!parse(*j)) return RT_ERR_ARG;
  const int nc = j->ncomp >= 3 ? 3 : 1;  // stbi_load(.., 0): RGB for 3/4 components, else grey
  std::unique_ptr<rt_image_host> im(new rt_image_host);
  im->px.assign((size_t)j->width * j->height * nc + 1, 0);
  const int decode_n = j->ncomp;
  struct Res {
    int hs, vs, ystep, ypos, wlo;
    const uint8_t *line0, *line1;
    std::vector<uint8_t> buf;
  } rs[4];
  for (int k = 0; k < decode_n; ++k) {
    Comp& c = j->comp[k];
    Res& r = rs[k];
    r.hs = j->hmax / c.h;
    r.vs = j->vmax / c.v;
    r.ystep = r.vs >> 1;
    r.wlo = (j->width + r.hs - 1) / r.hs;
    r.ypos = 0;
    r.line0 = r.line1 = c.plane.data();
    r.buf.assign((size_t)j->width + 3 + 8, 0);
  }
  const bool is_rgb = j->ncomp == 3 && (j->adobe_rgb || (j->app14_transform == 0 && !j->jfif));
  for (int y = 0; y < j->height; ++y) {
    const uint8_t* row[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int k = 0; k < decode_n; ++k) {
      Res& r = rs[k];
      const bool ybot = r.ystep >= (r.vs >> 1);
      const uint8_t* nr = ybot ? r.line1 : r.line0;
      const uint8_t* fr = ybot ? r.line0 : r.line1;
      if (r.hs == 1 && r.vs == 1) row[k] = row_1(r.buf.data(), nr, fr, r.wlo);
      else if (r.hs == 1 && r.vs == 2) row[k] = row_v2(r.buf.data(), nr, fr, r.wlo);
      else if (r.hs == 2 && r.vs == 1) row[k] = row_h2(r.buf.data(), nr, fr, r.wlo);
      else if (r.hs == 2 && r.vs == 2) row[k] = row_hv2(r.buf.data(), nr, fr, r.wlo);
      else row[k] = row_generic(r.buf.data(), nr, fr, r.wlo, r.hs);
      if (++r.ystep >= r.vs) {
        r.ystep = 0;
        r.line0 = r.line1;
        if (++r.ypos < j->comp[k].y) r.line1 += j->comp[k].w2;
      }
    }
    uint8_t* o = im->px.data() + (size_t)nc * j->width * y;
    if (nc == 3) {
      if (is_rgb) {
        for (int i = 0; i < j->width; ++i, o += 3) {
          o[0] = row[0][i];
          o[1] = row[1][i];
          o[2] = row[2][i];
        }
      } else {
        ycbcr_row(o, row[0], row[1], row[2], j->width, 3);
      }
    } else {
      memcpy(o, row[0], (size_t)j->width);
    }
  }
  im->px.resize((size_t)j->width * j->height * nc);
  im->view.width = j->width;
  im->view.height = j->height;
  im->view.bytes_per_pixel = nc;
  im->view.data = im->px.data();
  *out = im.release();
  return RT_OK;
}

int rt_image_load(const char* path, rt_image_host** out) {
  if (!path || !out) return RT_ERR_ARG;
  std::ifstream f(path, std::ios::binary);
  if (!f) return RT_ERR_ARG;
  std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  return rt_image_decode(bytes.data(), (int64_t)bytes.size(), out);
}

const rt_image_asset* rt_image_view(const rt_image_host* im) { return im ? &im->view : nullptr; }

void rt_image_free(rt_image_host* im) { delete im; }

}  // extern "C"
