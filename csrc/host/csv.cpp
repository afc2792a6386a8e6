// Host runtime: quote-aware CSV tokenizer + Spark-style schema inference + typed column parsing,
// dictionary encoding of string columns, and a multi-threaded word counter (the local[N] CPU
// executor of the wordcount config).
//
// Replaces Spark's univocity CSV reader with inferSchema (spark_workload_to_cloud_k8s.py:48) and the
// reference TF loader's csv.DictReader scan (train_tf_ps.py:75-149). RFC-4180 quoting: fields may
// be wrapped in double quotes, embedded quotes are doubled, quoted fields may contain delimiters
// and newlines (health.csv has quoted commas in `source`).
//
// Every entry point returns 0 on success (a negative code on error) and writes results through
// caller-provided buffers (two-call sizing pattern from Python/ctypes).
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

// Scan records: returns row starts (after the header if skip_header). Newlines inside quotes do not
// end a record. Trailing empty line ignored.
long scan_rows(const char* b, long n, long* starts, long max_rows, int* max_cols, char delim) {
  long rows = 0;
  long i = 0;
  int cols = 1, best = 0;
  bool inq = false;
  long rec_start = 0;
  bool any = false;
  while (i < n) {
    const char c = b[i];
    if (inq) {
      if (c == '"') {
        if (i + 1 < n && b[i + 1] == '"') { i += 2; continue; }
        inq = false;
      }
      ++i;
      continue;
    }
    if (c == '"') { inq = true; any = true; ++i; continue; }
    if (c == delim) { ++cols; any = true; ++i; continue; }
    if (c == '\n' || c == '\r') {
      if (any || i > rec_start) {
        if (starts && rows < max_rows) starts[rows] = rec_start;
        ++rows;
        best = std::max(best, cols);
      }
      if (c == '\r' && i + 1 < n && b[i + 1] == '\n') ++i;
      ++i;
      rec_start = i; cols = 1; any = false;
      continue;
    }
    any = true;
    ++i;
  }
  if (rec_start < n && (any || i > rec_start)) {
    if (starts && rows < max_rows) starts[rows] = rec_start;
    ++rows;
    best = std::max(best, cols);
  }
  if (max_cols) *max_cols = best;
  return rows;
}

inline bool is_space(char c) { return c == ' ' || c == '\t'; }

bool parse_i64(const char* s, int len, long long* out) {
  while (len > 0 && is_space(*s)) { ++s; --len; }
  while (len > 0 && is_space(s[len - 1])) --len;
  if (len <= 0 || len > 20) return false;
  char tmp[32];
  memcpy(tmp, s, len);
  tmp[len] = 0;
  char* end = nullptr;
  errno = 0;
  const long long v = strtoll(tmp, &end, 10);
  if (errno != 0 || end != tmp + len) return false;
  *out = v;
  return true;
}

bool parse_f64(const char* s, int len, double* out) {
  while (len > 0 && is_space(*s)) { ++s; --len; }
  while (len > 0 && is_space(s[len - 1])) --len;
  if (len <= 0 || len > 63) return false;
  char tmp[64];
  memcpy(tmp, s, len);
  tmp[len] = 0;
  if (!strcmp(tmp, "NaN") || !strcmp(tmp, "nan")) { *out = NAN; return true; }
  if (!strcmp(tmp, "Infinity") || !strcmp(tmp, "inf")) { *out = INFINITY; return true; }
  if (!strcmp(tmp, "-Infinity") || !strcmp(tmp, "-inf")) { *out = -INFINITY; return true; }
  char* end = nullptr;
  const double v = strtod(tmp, &end);
  if (end != tmp + len) return false;
  *out = v;
  return true;
}

bool parse_bool(const char* s, int len, bool* out) {
  if (len == 4 && !strncasecmp(s, "true", 4)) { *out = true; return true; }
  if (len == 5 && !strncasecmp(s, "false", 5)) { *out = false; return true; }
  return false;
}

// unescape a quoted field body ("" -> ") into dst; returns length
int unescape(const char* s, int len, bool quoted, char* dst) {
  if (!quoted) { memcpy(dst, s, len); return len; }
  int o = 0;
  for (int i = 0; i < len; ++i) {
    dst[o++] = s[i];
    if (s[i] == '"' && i + 1 < len && s[i + 1] == '"') ++i;
  }
  return o;
}

}  // namespace

extern "C" {

int ptgh_version() { return 1; }

// Count (starts == nullptr) or fill record start offsets.
int ptgh_csv_index(const char* buf, long len, int delim, long* nrows_out, int* ncols_out, long* starts, long max_rows) {
  int mc = 0;
  const long r = scan_rows(buf, len, starts, max_rows, &mc, (char)delim);
  if (nrows_out) *nrows_out = r;
  if (ncols_out) *ncols_out = mc;
  return 0;
}

// Field spans for rows [row_starts], ncols columns. Missing trailing fields: flen = -1.
// Empty unquoted field: flen = 0 (null in Spark semantics). fquoted marks quoted fields.
int ptgh_csv_fields(const char* buf, long len, const long* starts, long nrows, int ncols, int delim, long* fstart,
                    int* flen, unsigned char* fquoted) {
  const char d = (char)delim;
  const int nth = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  auto work = [&](long r0, long r1) {
    for (long r = r0; r < r1; ++r) {
      long i = starts[r];
      const long end = (r + 1 < nrows) ? starts[r + 1] : len;
      int c = 0;
      while (c < ncols) {
        const long idx = r * ncols + c;
        if (i >= end || buf[i] == '\n' || buf[i] == '\r') {
          fstart[idx] = i; flen[idx] = (c == 0 && i >= end) ? -1 : (c == 0 ? 0 : -1);
          if (c > 0) flen[idx] = -1;
          fquoted[idx] = 0;
          ++c;
          for (; c < ncols; ++c) { fstart[r * ncols + c] = i; flen[r * ncols + c] = -1; fquoted[r * ncols + c] = 0; }
          break;
        }
        if (buf[i] == '"') {
          const long s = i + 1;
          long j = s;
          while (j < end) {
            if (buf[j] == '"') {
              if (j + 1 < end && buf[j + 1] == '"') { j += 2; continue; }
              break;
            }
            ++j;
          }
          fstart[idx] = s; flen[idx] = (int)(j - s); fquoted[idx] = 1;
          i = j + 1;
          while (i < end && buf[i] != d && buf[i] != '\n' && buf[i] != '\r') ++i;
        } else {
          const long s = i;
          while (i < end && buf[i] != d && buf[i] != '\n' && buf[i] != '\r') ++i;
          fstart[idx] = s; flen[idx] = (int)(i - s); fquoted[idx] = 0;
        }
        ++c;
        if (i < end && buf[i] == d) {
          ++i;
          if (c == ncols) break;
          if (c < ncols && (i >= end || buf[i] == '\n' || buf[i] == '\r')) {  // trailing empty field
            fstart[r * ncols + c] = i; flen[r * ncols + c] = 0; fquoted[r * ncols + c] = 0; ++c;
            for (; c < ncols; ++c) { fstart[r * ncols + c] = i; flen[r * ncols + c] = -1; fquoted[r * ncols + c] = 0; }
            break;
          }
        } else {
          for (; c < ncols; ++c) { fstart[r * ncols + c] = i; flen[r * ncols + c] = -1; fquoted[r * ncols + c] = 0; }
          break;
        }
      }
    }
  };
  std::vector<std::thread> ts;
  const long per = (nrows + nth - 1) / nth;
  for (int t = 0; t < nth; ++t) {
    const long r0 = t * per, r1 = std::min(nrows, r0 + per);
    if (r0 < r1) ts.emplace_back(work, r0, r1);
  }
  for (auto& t : ts) t.join();
  return 0;
}

// Spark-style type inference for one column over rows [0, nrows):
//   0 = integer (int32 range), 1 = long, 2 = double, 3 = boolean, 4 = string, 5 = all null
int ptgh_csv_infer(const char* buf, const long* fstart, const int* flen, const unsigned char* fquoted, long nrows,
                   int ncols, int col, int* type_out) {
  int t = 5;  // null
  for (long r = 0; r < nrows; ++r) {
    const long idx = r * ncols + col;
    const int l = flen[idx];
    if (l <= 0) continue;  // null / missing
    const char* s = buf + fstart[idx];
    long long iv; double dv; bool bv;
    int ft;
    if (parse_i64(s, l, &iv)) ft = (iv >= INT32_MIN && iv <= INT32_MAX) ? 0 : 1;
    else if (parse_f64(s, l, &dv)) ft = 2;
    else if (parse_bool(s, l, &bv)) ft = 3;
    else ft = 4;
    if (t == 5) t = ft;
    else if (t != ft) {
      const bool tn = t <= 2, fn = ft <= 2;
      if (tn && fn) t = std::max(t, ft);
      else t = 4;
    }
    if (t == 4) break;
  }
  *type_out = t;
  return 0;
}

// typed parse: kind 0 = int64, 1 = double, 2 = bool(u8); invalid/empty -> valid=0
int ptgh_csv_parse(const char* buf, const long* fstart, const int* flen, long nrows, int ncols, int col, int kind,
                   void* out, unsigned char* valid) {
  for (long r = 0; r < nrows; ++r) {
    const long idx = r * ncols + col;
    const int l = flen[idx];
    bool ok = false;
    if (l > 0) {
      const char* s = buf + fstart[idx];
      if (kind == 0) { long long v; ok = parse_i64(s, l, &v); ((long long*)out)[r] = ok ? v : 0; }
      else if (kind == 1) { double v; ok = parse_f64(s, l, &v); ((double*)out)[r] = ok ? v : NAN; }
      else { bool v; ok = parse_bool(s, l, &v); ((unsigned char*)out)[r] = ok && v; }
    } else {
      if (kind == 0) ((long long*)out)[r] = 0;
      else if (kind == 1) ((double*)out)[r] = NAN;
      else ((unsigned char*)out)[r] = 0;
    }
    valid[r] = ok ? 1 : 0;
  }
  return 0;
}

// Dictionary-encode a string column (first-occurrence order). codes[r] = -1 for null (empty
// unquoted or missing). dict_bytes/dict_off receive the unescaped dictionary; returns count in ndict.
int ptgh_csv_dict_encode(const char* buf, const long* fstart, const int* flen, const unsigned char* fquoted,
                         long nrows, int ncols, int col, int* codes, char* dict_bytes, long dict_cap,
                         long* dict_off, long max_dict, long* ndict_out, long* dict_bytes_used) {
  std::unordered_map<std::string, int> m;
  m.reserve(1024);
  long nb = 0, nd = 0;
  std::string tmp;
  for (long r = 0; r < nrows; ++r) {
    const long idx = r * ncols + col;
    const int l = flen[idx];
    if (l < 0 || (l == 0 && !fquoted[idx])) { codes[r] = -1; continue; }
    tmp.resize(l);
    const int ul = unescape(buf + fstart[idx], l, fquoted[idx] != 0, &tmp[0]);
    tmp.resize(ul);
    auto it = m.find(tmp);
    if (it != m.end()) { codes[r] = it->second; continue; }
    if (nd >= max_dict || nb + ul > dict_cap) return -2;
    memcpy(dict_bytes + nb, tmp.data(), ul);
    dict_off[nd] = nb;
    nb += ul;
    m.emplace(tmp, (int)nd);
    codes[r] = (int)nd;
    ++nd;
  }
  dict_off[nd] = nb;
  *ndict_out = nd;
  *dict_bytes_used = nb;
  return 0;
}

// Word count over a text buffer split on whitespace; nthreads chunks (local[N]) with per-thread
// hash maps merged at the end. Two-call: out_words == nullptr returns sizes only.
int ptgh_word_count(const char* buf, long len, int nthreads, char* out_words, long out_cap, long* out_off,
                    long long* out_counts, long max_words, long* nwords_out, long* bytes_out) {
  if (nthreads < 1) nthreads = 1;
  std::vector<long> cuts(nthreads + 1, len);
  cuts[0] = 0;
  for (int t = 1; t < nthreads; ++t) {
    long c = len * t / nthreads;
    while (c < len && !isspace((unsigned char)buf[c])) ++c;
    cuts[t] = std::max(c, cuts[t - 1]);
  }
  std::vector<std::unordered_map<std::string_view, long long>> maps(nthreads);
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) {
    ts.emplace_back([&, t] {
      auto& mp = maps[t];
      long i = cuts[t];
      const long e = cuts[t + 1];
      while (i < e) {
        while (i < e && isspace((unsigned char)buf[i])) ++i;
        const long s = i;
        while (i < e && !isspace((unsigned char)buf[i])) ++i;
        if (i > s) ++mp[std::string_view(buf + s, i - s)];
      }
    });
  }
  for (auto& t : ts) t.join();
  for (int t = 1; t < nthreads; ++t)
    for (auto& kv : maps[t]) maps[0][kv.first] += kv.second;
  std::vector<std::pair<std::string_view, long long>> items(maps[0].begin(), maps[0].end());
  std::sort(items.begin(), items.end(), [](const auto& a, const auto& b) {
    return a.second != b.second ? a.second > b.second : a.first < b.first;
  });
  long bytes = 0;
  for (auto& it : items) bytes += (long)it.first.size();
  *nwords_out = (long)items.size();
  *bytes_out = bytes;
  if (!out_words) return 0;
  if ((long)items.size() > max_words || bytes > out_cap) return -2;
  long o = 0;
  for (size_t k = 0; k < items.size(); ++k) {
    out_off[k] = o;
    memcpy(out_words + o, items[k].first.data(), items[k].first.size());
    o += (long)items[k].first.size();
    out_counts[k] = items[k].second;
  }
  out_off[items.size()] = o;
  return 0;
}

}  // extern "C"
