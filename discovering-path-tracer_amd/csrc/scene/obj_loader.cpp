#include "obj_loader.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>

namespace pt {
namespace {

inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

// tinyobj tryParseDouble (tiny_obj_loader.h:897-1028): decimal mantissa in a
// double (digits after the point weighted by a 0.1^k table), exponent applied
// as ldexp(m * 5^e, e).  Not strtod: the rounding differs in corner cases and
// the vertex floats must be the reference's.
bool parse_double(const char* s, const char* end, double* out) {
  if (s >= end) return false;
  double m = 0.0;
  int ex = 0;
  bool neg = false, eneg = false, lead_dot = false;
  const char* c = s;
  int n = 0;
  if (*c == '+' || *c == '-') {
    neg = (*c == '-');
    ++c;
    lead_dot = (c != end && *c == '.');
  } else if (*c == '.') {
    lead_dot = true;
  } else if (!is_digit(*c)) {
    return false;
  }
  if (!lead_dot) {
    for (; c != end && is_digit(*c); ++c, ++n) m = m * 10 + (int)(*c - '0');
    if (n == 0) return false;
  }
  if (c != end) {
    bool exp_part = false;
    if (*c == '.') {
      ++c;
      static const double kPow[8] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
      for (int k = 1; c != end && is_digit(*c); ++c, ++k) m += (int)(*c - '0') * (k < 8 ? kPow[k] : pow(10.0, -k));
      exp_part = (c != end) && (*c == 'e' || *c == 'E');
    } else {
      exp_part = (*c == 'e' || *c == 'E');
    }
    if (exp_part) {
      ++c;
      if (c != end && (*c == '+' || *c == '-')) {
        eneg = (*c == '-');
        ++c;
      } else if (!is_digit(*c)) {
        return false;
      }
      int digits = 0;
      for (; c != end && is_digit(*c); ++c, ++digits) {
        if (ex > 2147483647 / 10) return false;
        ex = ex * 10 + (int)(*c - '0');
      }
      if (digits == 0) return false;
      if (eneg) ex = -ex;
    }
  }
  const double mag = ex ? ldexp(m * pow(5.0, ex), ex) : m;
  *out = neg ? -mag : mag;
  return true;
}

// parseReal (:1030-1038): missing or malformed numbers become 0.
float next_real(const char** tok) {
  *tok += strspn(*tok, " \t");
  const char* end = *tok + strcspn(*tok, " \t\r");
  double v = 0.0;
  parse_double(*tok, end, &v);
  *tok = end;
  return (float)v;
}

// pnpoly point-in-polygon crossing test (tiny_obj_loader.h:1438-1450), in
// the same float evaluation order.
bool point_in_tri(const float* px, const float* py, float tx, float ty) {
  bool in = false;
  for (int i = 0, j = 2; i < 3; j = i++) {
    if (((py[i] > ty) != (py[j] > ty)) && (tx < (px[j] - px[i]) * (ty - py[i]) / (py[j] - py[i]) + px[i]))
      in = !in;
  }
  return in;
}

// tinyobj's built-in ear clipping for faces of 5+ corners
// (tiny_obj_loader.h:1740-1955, TINYOBJLOADER_USE_MAPBOX_EARCUT undefined as
// in the reference build): project on the two axes picked from the first
// corner with a non-degenerate cross product, then repeatedly cut the ear at
// the current guess vertex — skipping reflex corners (cross * area < 0, area
// from the first two projected corners only, as tinyobj computes it) and
// corners whose triangle contains another remaining vertex — and finally
// emit the last three.  A face it cannot finish keeps only the ears found.
void ear_clip(const std::vector<int>& face, const float* v, std::vector<uint32_t>* tris) {
  const size_t n = face.size();
  int ax0 = 1, ax1 = 2;
  for (size_t k = 0; k < n; ++k) {
    const float* a = v + 3 * face[k % n];
    const float* b = v + 3 * face[(k + 1) % n];
    const float* c = v + 3 * face[(k + 2) % n];
    const float e0x = b[0] - a[0], e0y = b[1] - a[1], e0z = b[2] - a[2];
    const float e1x = c[0] - b[0], e1y = c[1] - b[1], e1z = c[2] - b[2];
    const float cx = fabsf(e0y * e1z - e0z * e1y);
    const float cy = fabsf(e0z * e1x - e0x * e1z);
    const float cz = fabsf(e0x * e1y - e0y * e1x);
    const float eps = 1.19209290e-07f;   // numeric_limits<float>::epsilon()
    if (cx > eps || cy > eps || cz > eps) {
      if (!(cx > cy && cx > cz)) {
        ax0 = 0;
        if (cz > cx && cz > cy) ax1 = 1;
      }
      break;
    }
  }
  std::vector<int> rem = face;
  size_t guess = 0, left = n, prev = n;
  while (rem.size() > 3 && left > 0) {
    const size_t m = rem.size();
    if (guess >= m) guess -= m;
    if (prev != m) {
      prev = m;
      left = m;
    } else {
      --left;
    }
    int ind[3];
    float px[3], py[3];
    for (int k = 0; k < 3; ++k) {
      ind[k] = rem[(guess + k) % m];
      px[k] = v[3 * ind[k] + ax0];
      py[k] = v[3 * ind[k] + ax1];
    }
    const float cross = (px[1] - px[0]) * (py[2] - py[1]) - (py[1] - py[0]) * (px[2] - px[1]);
    const float area = (px[0] * py[1] - py[0] * px[1]) * 0.5f;
    if (cross * area < 0.0f) {   // reflex corner
      ++guess;
      continue;
    }
    bool overlap = false;
    for (size_t o = 3; o < m && !overlap; ++o) {
      const int w = rem[(guess + o) % m];
      overlap = point_in_tri(px, py, v[3 * w + ax0], v[3 * w + ax1]);
    }
    if (overlap) {
      ++guess;
      continue;
    }
    tris->insert(tris->end(), {(uint32_t)ind[0], (uint32_t)ind[1], (uint32_t)ind[2]});
    rem.erase(rem.begin() + (long)((guess + 1) % m));
  }
  if (rem.size() == 3) tris->insert(tris->end(), {(uint32_t)rem[0], (uint32_t)rem[1], (uint32_t)rem[2]});
}

}  // namespace

int parse_obj(const char* text, size_t len, ObjScene* out, std::string* err) {
  *out = ObjScene();
  std::map<std::string, int> materials;   // no .mtl loading: every usemtl is unknown -> id -1
  int material = -1;
  bool in_shape = false;
  size_t pos = 0, line_no = 0;
  std::vector<int> face;
  std::string line;
  while (pos < len) {
    const char* nl = (const char*)memchr(text + pos, '\n', len - pos);
    size_t e = nl ? (size_t)(nl - text) : len;
    line.assign(text + pos, e - pos);
    pos = e + 1;
    ++line_no;
    const char* t = line.c_str();
    t += strspn(t, " \t");
    if (t[0] == 'v' && (t[1] == ' ' || t[1] == '\t')) {
      t += 2;
      const float x = next_real(&t), y = next_real(&t), z = next_real(&t);
      out->vertices.insert(out->vertices.end(), {x, y, z});
    } else if (t[0] == 'v' && t[1] == 't' && (t[2] == ' ' || t[2] == '\t')) {
      t += 3;
      const float u = next_real(&t), v = next_real(&t);
      out->texcoords.insert(out->texcoords.end(), {u, v});
    } else if ((t[0] == 'o' || t[0] == 'g') && (t[1] == ' ' || t[1] == '\t' || t[1] == 0 || t[1] == '\r')) {
      in_shape = true;
      ++out->shapes;
    } else if (strncmp(t, "usemtl", 6) == 0 && (t[6] == ' ' || t[6] == '\t')) {
      material = -1;
    } else if (t[0] == 'f' && (t[1] == ' ' || t[1] == '\t')) {
      if (!in_shape) { in_shape = true; ++out->shapes; }
      t += 2;
      const long nv = (long)(out->vertices.size() / 3);
      face.clear();
      for (;;) {
        t += strspn(t, " \t");
        if (*t == 0 || *t == '\r') break;
        char* endp;
        const long i = strtol(t, &endp, 10);
        if (endp == t || i == 0) {
          if (err) *err = "malformed face corner at line " + std::to_string(line_no);
          return -2;
        }
        face.push_back((int)(i > 0 ? i - 1 : nv + i));   // fixIndex: negative = relative
        t = endp;
        while (*t && *t != ' ' && *t != '\t' && *t != '\r') ++t;   // skip /vt/vn
      }
      const uint32_t mat = material >= 0 ? (uint32_t)material : 0u;
      if (face.size() < 3) continue;                              // :1500-1506 degenerate
      for (int vi : face) {
        if (vi < 0 || vi >= nv) {
          if (err) *err = "face vertex index out of range at line " + std::to_string(line_no);
          return -2;
        }
      }
      if (face.size() == 3) {
        out->indices.insert(out->indices.end(), {(uint32_t)face[0], (uint32_t)face[1], (uint32_t)face[2]});
        out->materialIds.push_back(mat);
      } else if (face.size() == 4) {                              // :1509-1604
        const float* v = out->vertices.data();
        const size_t a = face[0], b = face[1], c = face[2], d = face[3];
        const float e02x = v[c * 3 + 0] - v[a * 3 + 0], e02y = v[c * 3 + 1] - v[a * 3 + 1],
                    e02z = v[c * 3 + 2] - v[a * 3 + 2];
        const float e13x = v[d * 3 + 0] - v[b * 3 + 0], e13y = v[d * 3 + 1] - v[b * 3 + 1],
                    e13z = v[d * 3 + 2] - v[b * 3 + 2];
        const float s02 = e02x * e02x + e02y * e02y + e02z * e02z;
        const float s13 = e13x * e13x + e13y * e13y + e13z * e13z;
        if (s02 < s13)
          out->indices.insert(out->indices.end(), {(uint32_t)a, (uint32_t)b, (uint32_t)c, (uint32_t)a, (uint32_t)c, (uint32_t)d});
        else
          out->indices.insert(out->indices.end(), {(uint32_t)a, (uint32_t)b, (uint32_t)d, (uint32_t)b, (uint32_t)c, (uint32_t)d});
        out->materialIds.insert(out->materialIds.end(), {mat, mat});
      } else {                                                    // :1740-1955
        const size_t before = out->indices.size();
        ear_clip(face, out->vertices.data(), &out->indices);
        out->materialIds.insert(out->materialIds.end(), (out->indices.size() - before) / 3, mat);
      }
    }
  }
  return 0;
}

int load_obj_file(const std::string& path, ObjScene* out, std::string* err) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) {
    if (err) *err = "cannot open " + path;
    return -1;
  }
  std::string buf;
  char tmp[1 << 16];
  size_t n;
  while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) buf.append(tmp, n);
  fclose(f);
  return parse_obj(buf.data(), buf.size(), out, err);
}

}  // namespace pt
