// F1: native reader for the DLC / Lightning-Pose prediction CSVs on either
// side of the smoother (the on-disk format of the reference's scripts:
// scripts/multicam_example.py:83-92, scripts/pupil_example.py:63-72, read
// there with pd.read_csv(header=[0, 1, 2], index_col=0)).
//
// Layout of such a file: `header_rows` header lines (scorer / bodyparts /
// coords), then one line per frame: an index field followed by `cols`
// numeric fields.  The reader memory-maps the file, splits the data lines
// into contiguous blocks, one per thread, and parses every field with a
// correctly rounded decimal conversion (Clinger fast path, strtod_l
// otherwise -- the result of pandas' float_precision="round_trip").  Empty
// fields and pandas' default NA strings become NaN.
// Output is row-major float64 (rows, cols) without the index column; the
// header lines are returned verbatim for the Python side to split.
//
// Host-only code (compiled by g++, linked into libeks_hip.so).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <clocale>
#include <locale.h>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

#include "../../include/eks_io.h"

namespace {

thread_local std::string g_io_err;

int io_err(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_io_err = buf;
  return code;
}

struct Mapped {
  const char *p = nullptr;
  size_t n = 0;
  int fd = -1;
  ~Mapped() {
    if (p && n) munmap((void *)p, n);
    if (fd >= 0) close(fd);
  }
  bool open_file(const char *path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    n = (size_t)st.st_size;
    if (n == 0) return true;
    void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      n = 0;
      return false;
    }
    madvise(m, n, MADV_SEQUENTIAL);
    p = (const char *)m;
    return true;
  }
};

// end of the line starting at s (position of '\n' or e)
inline const char *line_end(const char *s, const char *e) {
  const void *q = memchr(s, '\n', (size_t)(e - s));
  return q ? (const char *)q : e;
}

inline bool is_blank_line(const char *s, const char *le) {
  for (; s < le; ++s)
    if (*s != '\r' && *s != ' ' && *s != '\t') return false;
  return true;
}

// pandas' default NA strings (pandas.io.parsers STR_NA_VALUES)
bool is_na(const char *s, size_t n) {
  static const char *na[] = {"",     "#N/A", "#N/A N/A", "#NA", "-1.#IND", "-1.#QNAN", "-NaN",
                             "-nan", "1.#IND", "1.#QNAN", "<NA>", "N/A", "NA", "NULL", "NaN",
                             "None", "n/a",  "nan",  "null"};
  for (const char *x : na)
    if (strlen(x) == n && memcmp(x, s, n) == 0) return true;
  return false;
}

// strtod in the "C" locale, thread-safe (one locale object per process)
double strtod_c(const char *s, const char *t, bool &ok) {
  static locale_t c_loc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
  char buf[128];
  std::string big;
  const size_t n = (size_t)(t - s);
  const char *z;
  if (n < sizeof buf) {
    memcpy(buf, s, n);
    buf[n] = '\0';
    z = buf;
  } else {
    big.assign(s, t);
    z = big.c_str();
  }
  char *end = nullptr;
  const double v = strtod_l(z, &end, c_loc);
  ok = (end == z + n) && n > 0;
  return v;
}

// Decimal -> double.  Clinger's fast path (exact when the decimal mantissa
// fits in 53 bits and |power of ten| <= 22: one correctly rounded multiply
// or divide of two exact doubles) covers the pose-estimator outputs
// (<= 17 significant digits, small exponents); everything else goes to
// strtod_l.  Both are correctly rounded.  Returns false if [s, t) is not a
// complete number.
inline bool parse_number(const char *s, const char *t, double &v) {
  static const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                 1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  const char *c = s;
  bool neg = false;
  if (c < t && (*c == '-' || *c == '+')) neg = (*c++ == '-');
  uint64_t m = 0;
  int nd = 0, frac = 0;
  bool any = false;
  while (c < t && *c == '0') {
    ++c;
    any = true;
  }
  while (c < t && (unsigned)(*c - '0') < 10) {
    m = m * 10 + (uint64_t)(*c++ - '0');
    ++nd;
    any = true;
  }
  if (c < t && *c == '.') {
    ++c;
    if (nd == 0)
      while (c < t && *c == '0') {
        ++c;
        ++frac;
        any = true;
      }
    while (c < t && (unsigned)(*c - '0') < 10) {
      m = m * 10 + (uint64_t)(*c++ - '0');
      ++nd;
      ++frac;
      any = true;
    }
  }
  if (!any) {
    bool ok;
    v = strtod_c(s, t, ok);  // inf / nan spellings
    return ok;
  }
  int e10 = 0;
  if (c < t && (*c == 'e' || *c == 'E')) {
    ++c;
    bool eneg = false;
    if (c < t && (*c == '-' || *c == '+')) eneg = (*c++ == '-');
    if (c == t) return false;
    int e = 0;
    while (c < t && (unsigned)(*c - '0') < 10) {
      if (e < 100000) e = e * 10 + (*c - '0');
      ++c;
    }
    e10 = eneg ? -e : e;
  }
  if (c != t) return false;
  const int p = e10 - frac;
  if (nd <= 19 && m <= (1ULL << 53) && p >= -22 && p <= 22) {
    const double dm = (double)m;
    v = p < 0 ? dm / p10[-p] : dm * p10[p];
    if (neg) v = -v;
    return true;
  }
  // 16-19 significant digits (e.g. Python repr output): the quotient in x87
  // extended precision (64-bit mantissa; m and 10^|p| <= 10^27 are exact)
  // carries 11 guard bits; unless they sit within one unit of the halfway
  // pattern, rounding it to double gives the correctly rounded result.
  if (nd <= 19 && p >= -27 && p <= 27) {
    long double pw = 1.0L;
    for (int i = 0; i < (p < 0 ? -p : p); ++i) pw *= 10.0L;
    const long double x = p < 0 ? (long double)m / pw : (long double)m * pw;
    int ex;
    const long double fr = frexpl(x, &ex);  // [0.5, 1)
    const uint64_t bits = (uint64_t)ldexpl(fr, 64);
    const int low = (int)(bits & 0x7FF);
    if (low < 0x3FF || low > 0x401) {
      v = (double)x;
      if (neg) v = -v;
      return true;
    }
  }
  bool ok;
  v = strtod_c(s, t, ok);
  return ok;
}

// parse one field [s, t) into v; false if it is not a number or NA
inline bool parse_field(const char *s, const char *t, double &v) {
  while (s < t && (*s == ' ' || *s == '\t')) ++s;
  while (t > s && (t[-1] == ' ' || t[-1] == '\t' || t[-1] == '\r')) --t;
  if (s < t && *s == '"' && t - s >= 2 && t[-1] == '"') {
    ++s;
    --t;
  }
  if (s == t) {
    v = std::numeric_limits<double>::quiet_NaN();
    return true;
  }
  if (parse_number(s, t, v)) return true;
  if (is_na(s, (size_t)(t - s))) {
    v = std::numeric_limits<double>::quiet_NaN();
    return true;
  }
  return false;
}

inline int64_t count_fields(const char *s, const char *le) {
  int64_t k = 1;
  for (; s < le; ++s) k += (*s == ',');
  return k;
}

// header: first `header_rows` lines; data starts after them
bool split_header(const char *p, const char *e, int header_rows, const char *&data,
                  size_t &header_len) {
  const char *s = p;
  for (int h = 0; h < header_rows; ++h) {
    if (s >= e) return false;
    const char *le = line_end(s, e);
    s = le < e ? le + 1 : e;
  }
  data = s;
  header_len = (size_t)(s - p);
  return true;
}

}  // namespace

extern "C" {

const char *eks_io_last_error(void) { return g_io_err.c_str(); }

int eks_csv_probe(const char *path, int header_rows, int64_t *rows, int64_t *cols,
                  int64_t *header_bytes) {
  g_io_err.clear();
  if (!path || !rows || !cols || header_rows < 0)
    return io_err(EKS_IO_ERR_ARG, "eks_csv_probe: bad argument");
  Mapped m;
  if (!m.open_file(path)) return io_err(EKS_IO_ERR_FILE, "cannot open %s", path);
  const char *p = m.p, *e = m.p + m.n;
  const char *data;
  size_t hl = 0;
  if (!split_header(p, e, header_rows, data, hl))
    return io_err(EKS_IO_ERR_FORMAT, "%s: fewer than %d header lines", path, header_rows);
  int64_t nr = 0, nc = -1;
  for (const char *s = data; s < e;) {
    const char *le = line_end(s, e);
    if (!is_blank_line(s, le)) {
      if (nc < 0) nc = count_fields(s, le) - 1;
      ++nr;
    }
    s = le + 1;
  }
  *rows = nr;
  *cols = nc < 0 ? 0 : nc;
  if (header_bytes) *header_bytes = (int64_t)hl + 1;
  return EKS_IO_OK;
}

int eks_csv_read(const char *path, int header_rows, double *data, int64_t rows, int64_t cols,
                 double *index, char *header, int64_t header_bytes, int nthreads) {
  g_io_err.clear();
  if (!path || (!data && rows * cols > 0) || header_rows < 0 || rows < 0 || cols < 0)
    return io_err(EKS_IO_ERR_ARG, "eks_csv_read: bad argument");
  Mapped m;
  if (!m.open_file(path)) return io_err(EKS_IO_ERR_FILE, "cannot open %s", path);
  const char *p = m.p, *e = m.p + m.n;
  const char *d0;
  size_t hl = 0;
  if (!split_header(p, e, header_rows, d0, hl))
    return io_err(EKS_IO_ERR_FORMAT, "%s: fewer than %d header lines", path, header_rows);
  if (header) {
    if (header_bytes < (int64_t)hl + 1)
      return io_err(EKS_IO_ERR_ARG, "eks_csv_read: header buffer too small (%lld < %zu)",
                    (long long)header_bytes, hl + 1);
    memcpy(header, p, hl);
    header[hl] = '\0';
  }
  // block boundaries at line starts, ~equal bytes per thread
  const size_t body = (size_t)(e - d0);
  int nt = nthreads > 0 ? nthreads : (int)std::min<unsigned>(16, std::thread::hardware_concurrency());
  nt = std::max(1, std::min<int>(nt, (int)(body / (1 << 16)) + 1));
  std::vector<const char *> cut(nt + 1);
  cut[0] = d0;
  cut[nt] = e;
  for (int i = 1; i < nt; ++i) {
    const char *s = d0 + body * i / nt;
    if (s < cut[i - 1]) s = cut[i - 1];
    const char *le = line_end(s, e);
    cut[i] = le < e ? le + 1 : e;
  }
  // pass 1: non-blank lines per block -> row offsets
  std::vector<int64_t> cnt(nt, 0);
  auto count_block = [&](int i) {
    int64_t c = 0;
    for (const char *s = cut[i]; s < cut[i + 1];) {
      const char *le = line_end(s, cut[i + 1]);
      if (!is_blank_line(s, le)) ++c;
      s = le + 1;
    }
    cnt[i] = c;
  };
  std::vector<std::thread> th;
  for (int i = 1; i < nt; ++i) th.emplace_back(count_block, i);
  count_block(0);
  for (auto &t : th) t.join();
  th.clear();
  std::vector<int64_t> off(nt + 1, 0);
  for (int i = 0; i < nt; ++i) off[i + 1] = off[i] + cnt[i];
  if (off[nt] != rows)
    return io_err(EKS_IO_ERR_FORMAT, "%s: %lld data rows, caller expected %lld", path,
                  (long long)off[nt], (long long)rows);
  // pass 2: parse
  std::atomic<int64_t> bad_row{-1};
  std::atomic<int> bad_kind{0};
  auto parse_block = [&](int i) {
    int64_t r = off[i];
    for (const char *s = cut[i]; s < cut[i + 1];) {
      const char *le = line_end(s, cut[i + 1]);
      if (is_blank_line(s, le)) {
        s = le + 1;
        continue;
      }
      const char *f = s;
      const char *c = (const char *)memchr(f, ',', (size_t)(le - f));
      if (!c) c = le;
      double v;
      if (index) index[r] = parse_field(f, c, v) ? v : std::numeric_limits<double>::quiet_NaN();
      int64_t j = 0;
      f = c + 1;
      double *row = data + r * cols;
      while (c < le && j < cols) {
        c = (const char *)memchr(f, ',', (size_t)(le - f));
        if (!c) c = le;
        if (!parse_field(f, c, row[j])) {
          bad_row.store(r);
          bad_kind.store(1);
          return;
        }
        ++j;
        f = c + 1;
      }
      if (j != cols || c < le) {
        bad_row.store(r);
        bad_kind.store(2);
        return;
      }
      ++r;
      s = le + 1;
    }
  };
  for (int i = 1; i < nt; ++i) th.emplace_back(parse_block, i);
  parse_block(0);
  for (auto &t : th) t.join();
  if (bad_row.load() >= 0)
    return io_err(EKS_IO_ERR_FORMAT, "%s: data row %lld: %s", path, (long long)bad_row.load(),
                  bad_kind.load() == 1 ? "non-numeric field" : "wrong number of fields");
  return EKS_IO_OK;
}

}  // extern "C"
