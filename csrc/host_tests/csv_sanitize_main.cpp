// Sanitizer driver for the host C++ runtime: csrc/host/csv.cpp is compiled together
// with this file under -fsanitize=address,undefined into a standalone executable (no Python, no
// preload), then every entry point runs over (1) the CSV files named on the command line and
// (2) seeded random fuzz buffers full of quotes, delimiters, CR/LF and ragged rows.  Any heap /
// stack overflow, use-after-free or UB aborts the process with the sanitizer's report.
// Built and run by tests/test_host_sanitize_cpu.py.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

extern "C" {
int ptgh_csv_index(const char* buf, long len, int delim, long* nrows_out, int* ncols_out, long* starts, long max_rows);
int ptgh_csv_fields(const char* buf, long len, const long* starts, long nrows, int ncols, int delim, long* fstart,
                    int* flen, unsigned char* fquoted);
int ptgh_csv_infer(const char* buf, const long* fstart, const int* flen, const unsigned char* fquoted, long nrows,
                   int ncols, int col, int* type_out);
int ptgh_csv_parse(const char* buf, const long* fstart, const int* flen, long nrows, int ncols, int col, int kind,
                   void* out, unsigned char* valid);
int ptgh_csv_dict_encode(const char* buf, const long* fstart, const int* flen, const unsigned char* fquoted,
                         long nrows, int ncols, int col, int* codes, char* dict_bytes, long dict_cap,
                         long* dict_off, long max_dict, long* ndict_out, long* dict_bytes_used);
int ptgh_word_count(const char* buf, long len, int nthreads, char* out_words, long out_cap, long* out_off,
                    long long* out_counts, long max_words, long* nwords_out, long* bytes_out);
}

static long g_cells = 0, g_words = 0;

// Exact-size heap copies so ASan sees any read past the end of the caller's buffer.
static void run_csv(const std::string& text, int delim) {
  const long len = (long)text.size();
  char* buf = (char*)malloc(len ? len : 1);
  memcpy(buf, text.data(), len);
  long nrows = 0;
  int ncols = 0;
  ptgh_csv_index(buf, len, delim, &nrows, &ncols, nullptr, 0);
  std::vector<long> starts(nrows ? nrows : 1);
  long n2 = 0;
  int c2 = 0;
  ptgh_csv_index(buf, len, delim, &n2, &c2, starts.data(), nrows);
  if (n2 != nrows || c2 != ncols) { fprintf(stderr, "index count mismatch\n"); exit(2); }
  if (nrows && ncols) {
    const long cells = nrows * (long)ncols;
    long* fstart = (long*)malloc(cells * sizeof(long));
    int* flen = (int*)malloc(cells * sizeof(int));
    unsigned char* fq = (unsigned char*)malloc(cells);
    ptgh_csv_fields(buf, len, starts.data(), nrows, ncols, delim, fstart, flen, fq);
    for (long i = 0; i < cells; ++i) {
      if (flen[i] > 0 && (fstart[i] < 0 || fstart[i] + flen[i] > len)) { fprintf(stderr, "field out of range\n"); exit(3); }
    }
    for (int c = 0; c < ncols; ++c) {
      int t = -1;
      ptgh_csv_infer(buf, fstart, flen, fq, nrows, ncols, c, &t);
      std::vector<long long> iv(nrows);
      std::vector<double> dv(nrows);
      std::vector<unsigned char> bv(nrows), valid(nrows);
      ptgh_csv_parse(buf, fstart, flen, nrows, ncols, c, 0, iv.data(), valid.data());
      ptgh_csv_parse(buf, fstart, flen, nrows, ncols, c, 1, dv.data(), valid.data());
      ptgh_csv_parse(buf, fstart, flen, nrows, ncols, c, 2, bv.data(), valid.data());
      std::vector<int> codes(nrows);
      const long cap = len + 1, maxd = nrows + 1;
      char* dict = (char*)malloc(cap);
      long* doff = (long*)malloc((maxd + 1) * sizeof(long));
      long nd = 0, used = 0;
      ptgh_csv_dict_encode(buf, fstart, flen, fq, nrows, ncols, c, codes.data(), dict, cap, doff, maxd, &nd, &used);
      // a too-small dictionary must be refused, not overrun
      long nd2 = 0, used2 = 0;
      ptgh_csv_dict_encode(buf, fstart, flen, fq, nrows, ncols, c, codes.data(), dict, 1, doff, 1, &nd2, &used2);
      free(dict);
      free(doff);
    }
    g_cells += cells;
    free(fstart);
    free(flen);
    free(fq);
  }
  for (int th : {1, 3}) {
    long nw = 0, nb = 0;
    ptgh_word_count(buf, len, th, nullptr, 0, nullptr, nullptr, 0, &nw, &nb);
    char* words = (char*)malloc(nb ? nb : 1);
    long* off = (long*)malloc((nw + 1) * sizeof(long));
    long long* cnt = (long long*)malloc((nw ? nw : 1) * sizeof(long long));
    long nw2 = 0, nb2 = 0;
    if (ptgh_word_count(buf, len, th, words, nb, off, cnt, nw, &nw2, &nb2) != 0) { fprintf(stderr, "wc\n"); exit(4); }
    g_words += nw;
    free(words);
    free(off);
    free(cnt);
  }
  free(buf);
}

static std::string read_file(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) { fprintf(stderr, "cannot open %s\n", path); exit(5); }
  std::string s;
  char tmp[65536];
  size_t k;
  while ((k = fread(tmp, 1, sizeof tmp, f)) > 0) s.append(tmp, k);
  fclose(f);
  return s;
}

int main(int argc, char** argv) {
  int fuzz = 400;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--fuzz") && i + 1 < argc) { fuzz = atoi(argv[++i]); continue; }
    run_csv(read_file(argv[i]), ',');
  }
  std::mt19937_64 rng(12345);
  const char alphabet[] = "ab1.5-e\",\n\r\t ;xyz\"\"9TrueFALSE";
  for (int it = 0; it < fuzz; ++it) {
    const int n = (int)(rng() % 600);
    std::string s;
    s.reserve(n);
    for (int j = 0; j < n; ++j) s.push_back(alphabet[rng() % (sizeof(alphabet) - 1)]);
    run_csv(s, (it & 1) ? ';' : ',');
  }
  run_csv("", ',');
  run_csv("\"", ',');
  run_csv("a,b\n\"unterminated,1\n", ',');
  printf("SANITIZE_OK cells=%ld words=%ld\n", g_cells, g_words);
  return 0;
}
