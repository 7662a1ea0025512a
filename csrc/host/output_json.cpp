// output_json.cpp — native renderer of the reference's per-batch result file.
//
// Reference (worker.py:1580-1581, models.py:109-126): every batch ends in
// ``json.dump(results, f, indent=4, cls=NpEncoder)`` of
//   {"<img>.jpeg": [[["<wnid>", "<label>", <prob>] x 5]], "<bad>.jpeg": "Failed to download file from SDFS"}
// CPython's pure-Python indent encoder runs ~29k images/s on one core, a third of
// one MI355X's output rate. This renders the byte-identical document in C++:
// the per-class strings ("wnid",\n<indent>"label",\n<indent>) are pre-rendered
// once by the caller, so an image costs five table copies and five float
// formats. Floats follow Python's repr exactly: the shortest round-trip digits
// (std::to_chars), fixed notation for decimal exponents -4 <= e < 16, else
// d.ddde+XX (two exponent digits at least), ".0" appended to integral values.
// Called through ctypes, which releases the GIL: the writer threads of a rank
// render concurrently with its serve loop.
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace {

struct Out {
  char* p;
  char* end;
  bool ok = true;
  void put(const char* s, size_t n) {
    if (!ok || (size_t)(end - p) < n) {
      ok = false;
      return;
    }
    std::memcpy(p, s, n);
    p += n;
  }
  void put(const char* s) { put(s, std::strlen(s)); }
};

// Python repr(float) (float_repr_style 'short', Py_DTSF_ADD_DOT_0)
int py_repr(double v, char* buf) {
  if (std::isnan(v)) return std::sprintf(buf, "NaN");  // json.dumps(allow_nan=True)
  if (std::isinf(v)) return std::sprintf(buf, v > 0 ? "Infinity" : "-Infinity");
  char sci[64];
  auto r = std::to_chars(sci, sci + sizeof(sci), v, std::chars_format::scientific);
  *r.ptr = 0;
  char* q = sci;
  int n = 0;
  if (*q == '-') {
    buf[n++] = '-';
    ++q;
  }
  char digits[40];
  int nd = 0;
  for (; *q && *q != 'e'; ++q)
    if (*q != '.') digits[nd++] = *q;
  const int exp10 = std::atoi(q + 1);  // value = d.ddd * 10^exp10
  while (nd > 1 && digits[nd - 1] == '0') --nd;
  const int decpt = exp10 + 1;         // value = 0.ddd * 10^decpt
  if (decpt <= -4 || decpt > 16) {     // exponent form: d[.ddd]e+XX
    buf[n++] = digits[0];
    if (nd > 1) {
      buf[n++] = '.';
      for (int i = 1; i < nd; ++i) buf[n++] = digits[i];
    }
    n += std::sprintf(buf + n, "e%c%02d", exp10 < 0 ? '-' : '+', exp10 < 0 ? -exp10 : exp10);
    return n;
  }
  if (decpt <= 0) {
    buf[n++] = '0';
    buf[n++] = '.';
    for (int i = 0; i < -decpt; ++i) buf[n++] = '0';
    for (int i = 0; i < nd; ++i) buf[n++] = digits[i];
  } else if (decpt < nd) {
    for (int i = 0; i < decpt; ++i) buf[n++] = digits[i];
    buf[n++] = '.';
    for (int i = decpt; i < nd; ++i) buf[n++] = digits[i];
  } else {
    for (int i = 0; i < nd; ++i) buf[n++] = digits[i];
    for (int i = nd; i < decpt; ++i) buf[n++] = '0';
    buf[n++] = '.';
    buf[n++] = '0';
  }
  return n;
}

}  // namespace

extern "C" {

// Render one batch document into out[0, cap). Returns the byte count, or -1 if
// cap is too small. Entry e (0 <= e < n) is the key keys[key_off[e], key_off[e+1])
// (already a JSON string literal, quotes included) with the top-k row
// rows[e] of top_idx / top_p ([rows][k], row-major), or the failure string when
// rows[e] < 0. cls: per-class pre-rendered text cls[cls_off[c], cls_off[c+1]);
// an out-of-range class id renders as class 0's text (never read past the table).
long dml_render_top5_json(int n, const char* keys, const long* key_off, const int* rows, const int* top_idx,
                          const float* top_p, int k, const char* cls, const long* cls_off, int ncls, char* out,
                          long cap) {
  static const char FAILED[] = "\"Failed to download file from SDFS\"";
  Out o{out, out + cap};
  if (n == 0) {
    o.put("{}");
    return o.ok ? (long)(o.p - out) : -1;
  }
  char num[64];
  o.put("{");
  for (int e = 0; e < n; ++e) {
    o.put(e ? ",\n    " : "\n    ");
    o.put(keys + key_off[e], (size_t)(key_off[e + 1] - key_off[e]));
    o.put(": ");
    const int r = rows[e];
    if (r < 0) {
      o.put(FAILED, sizeof(FAILED) - 1);
      continue;
    }
    o.put("[\n        [");
    for (int j = 0; j < k; ++j) {
      o.put(j ? ",\n            [\n                " : "\n            [\n                ");
      int c = top_idx[(long)r * k + j];
      if (c < 0 || c >= ncls) c = 0;
      o.put(cls + cls_off[c], (size_t)(cls_off[c + 1] - cls_off[c]));
      const int m = py_repr((double)top_p[(long)r * k + j], num);
      o.put(num, (size_t)m);
      o.put("\n            ]");
    }
    o.put("\n        ]\n    ]");
  }
  o.put("\n}");
  return o.ok ? (long)(o.p - out) : -1;
}

// Render and write one file (create/truncate) in one call; returns bytes written or -1.
long dml_write_top5_json(const char* path, int n, const char* keys, const long* key_off, const int* rows,
                         const int* top_idx, const float* top_p, int k, const char* cls, const long* cls_off,
                         int ncls, char* scratch, long cap) {
  const long len = dml_render_top5_json(n, keys, key_off, rows, top_idx, top_p, k, cls, cls_off, ncls, scratch, cap);
  if (len < 0) return -1;
  FILE* f = std::fopen(path, "wb");
  if (!f) return -1;
  const size_t w = std::fwrite(scratch, 1, (size_t)len, f);
  const int rc = std::fclose(f);
  return (w == (size_t)len && rc == 0) ? len : -1;
}

// repr of one double (tests compare it with Python's repr)
int dml_py_repr(double v, char* buf) { return py_repr(v, buf); }

}  // extern "C"
