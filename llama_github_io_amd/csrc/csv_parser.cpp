// Multi-threaded CSV tokenizer + per-cell type classifier (host runtime).
//
// Reference behaviour: h2o-core/src/main/java/water/parser/CsvParser.java (tokenizing, quotes, NA
// strings), ParseSetup.java (separator / header / column type guessing). Here: one pass finds record
// starts (quote aware, memchr-driven), then record ranges are parsed in parallel; every cell becomes
// a double (NaN if not numeric) plus a kind byte (0 = NA/empty, 1 = number, 2 = text) and, for text
// cells, its byte span in the input buffer (Python builds enum domains / strings from spans only for
// columns that need them).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Col {
  std::vector<double> num;
  std::vector<uint8_t> kind;
  std::vector<int64_t> off;
  std::vector<int32_t> len;
  std::atomic<int64_t> n_text{0};
  std::atomic<int64_t> n_num{0};
};

struct Result {
  int64_t nrows = 0;
  int ncols = 0;
  std::vector<std::string> header;
  std::vector<Col*> cols;
  ~Result() { for (auto* c : cols) delete c; }
};

const double kPow10[] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                         1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

inline bool is_na_token(const char* s, int n) {
  if (n == 0) return true;
  switch (n) {
    case 1: return s[0] == '?';
    case 2: return (s[0] == 'N' && s[1] == 'A');
    case 3: return (std::strncmp(s, "NaN", 3) == 0 || std::strncmp(s, "nan", 3) == 0 || std::strncmp(s, "N/A", 3) == 0);
    case 4: return std::strncmp(s, "null", 4) == 0 || std::strncmp(s, "NULL", 4) == 0 || std::strncmp(s, "None", 4) == 0;
    default: return false;
  }
}

// fast decimal parse; returns false if the token is not a number
inline bool parse_number(const char* s, int n, double* out) {
  const char* p = s;
  const char* e = s + n;
  while (p < e && (*p == ' ' || *p == '\t')) ++p;
  while (e > p && (e[-1] == ' ' || e[-1] == '\t' || e[-1] == '\r')) --e;
  if (p == e) return false;
  bool neg = false;
  if (*p == '+' || *p == '-') { neg = *p == '-'; ++p; }
  if (p == e) return false;
  if (e - p == 3 && (std::strncmp(p, "Inf", 3) == 0 || std::strncmp(p, "inf", 3) == 0)) {
    *out = neg ? -INFINITY : INFINITY; return true;
  }
  if (e - p == 8 && std::strncmp(p, "Infinity", 8) == 0) { *out = neg ? -INFINITY : INFINITY; return true; }
  uint64_t mant = 0;
  int digits = 0, exp10 = 0;
  bool any = false;
  while (p < e && *p >= '0' && *p <= '9') {
    if (digits < 19) { mant = mant * 10 + (*p - '0'); if (mant) ++digits; } else ++exp10;
    ++p; any = true;
  }
  if (p < e && *p == '.') {
    ++p;
    while (p < e && *p >= '0' && *p <= '9') {
      if (digits < 19) { mant = mant * 10 + (*p - '0'); if (mant) ++digits; --exp10; }
      ++p; any = true;
    }
  }
  if (!any) return false;
  if (p < e && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < e && (*p == '+' || *p == '-')) { eneg = *p == '-'; ++p; }
    if (p == e || !(*p >= '0' && *p <= '9')) return false;
    int ex = 0;
    while (p < e && *p >= '0' && *p <= '9') { if (ex < 100000) ex = ex * 10 + (*p - '0'); ++p; }
    exp10 += eneg ? -ex : ex;
  }
  if (p != e) return false;
  double v;
  if (digits <= 15 && exp10 >= -22 && exp10 <= 22) {
    v = (double)mant;
    v = exp10 >= 0 ? v * kPow10[exp10] : v / kPow10[-exp10];
  } else {
    std::string tmp(s, (size_t)n);
    char* endp = nullptr;
    v = std::strtod(tmp.c_str(), &endp);
    *out = v;
    return true;
  }
  *out = neg ? -v : v;
  return true;
}

// record starts, quote aware
std::vector<int64_t> find_records(const char* buf, int64_t len, char quote) {
  std::vector<int64_t> starts;
  starts.reserve(1 << 16);
  int64_t i = 0;
  // skip UTF-8 BOM
  if (len >= 3 && (uint8_t)buf[0] == 0xEF && (uint8_t)buf[1] == 0xBB && (uint8_t)buf[2] == 0xBF) i = 3;
  bool has_quote = quote && std::memchr(buf, quote, (size_t)len) != nullptr;
  starts.push_back(i);
  if (!has_quote) {
    while (i < len) {
      const char* nl = (const char*)std::memchr(buf + i, '\n', (size_t)(len - i));
      if (!nl) break;
      i = nl - buf + 1;
      if (i < len) starts.push_back(i);
    }
  } else {
    bool inq = false;
    for (; i < len; ++i) {
      const char c = buf[i];
      if (c == quote) inq = !inq;
      else if (c == '\n' && !inq && i + 1 < len) starts.push_back(i + 1);
    }
  }
  return starts;
}

// split one record into cells (spans); handles quotes ("" escape) — returns number of cells
inline int split_record(const char* buf, int64_t a, int64_t b, char sep, char quote,
                        std::vector<int64_t>& co, std::vector<int32_t>& cl, std::vector<uint8_t>& cq) {
  co.clear(); cl.clear(); cq.clear();
  while (b > a && (buf[b - 1] == '\n' || buf[b - 1] == '\r')) --b;
  if (b <= a) return 0;
  int64_t i = a;
  while (true) {
    if (quote && i < b && buf[i] == quote) {
      int64_t j = i + 1;
      uint8_t esc = 0;
      while (j < b) {
        if (buf[j] == quote) {
          if (j + 1 < b && buf[j + 1] == quote) { j += 2; esc = 1; continue; }
          break;
        }
        ++j;
      }
      co.push_back(i + 1); cl.push_back((int32_t)(j - i - 1)); cq.push_back(esc ? 2 : 1);
      i = j + 1;
      while (i < b && buf[i] != sep) ++i;
    } else {
      int64_t j = i;
      if (sep == ' ') {
        while (j < b && buf[j] != ' ' && buf[j] != '\t') ++j;
      } else {
        const char* hit = (const char*)std::memchr(buf + i, sep, (size_t)(b - i));
        j = hit ? hit - buf : b;
      }
      // trim spaces
      int64_t s = i, t = j;
      while (s < t && (buf[s] == ' ' || buf[s] == '\t')) ++s;
      while (t > s && (buf[t - 1] == ' ' || buf[t - 1] == '\t')) --t;
      co.push_back(s); cl.push_back((int32_t)(t - s)); cq.push_back(0);
      i = j;
    }
    if (i >= b) break;
    ++i;  // skip separator
    if (sep == ' ') while (i < b && (buf[i] == ' ' || buf[i] == '\t')) ++i;
    if (i >= b) { co.push_back(b); cl.push_back(0); cq.push_back(0); break; }
  }
  return (int)co.size();
}

}  // namespace

#include "abi.h"

extern "C" {

int h2o_abi_version() { return H2O_ABI_VERSION; }


char h2o_csv_guess_sep(const char* buf, int64_t len) {
  const char cands[] = {',', '\t', ';', '|', ' '};
  int64_t lim = std::min<int64_t>(len, 1 << 16);
  int best = 0;
  char bsep = ',';
  for (char c : cands) {
    // count per line over the first lines; prefer consistent non-zero counts
    int lines = 0, consistent = 0, first = -1;
    int64_t i = 0;
    int cnt = 0;
    bool inq = false;
    for (; i < lim && lines < 20; ++i) {
      if (buf[i] == '"') inq = !inq;
      if (!inq && buf[i] == c) ++cnt;
      if (buf[i] == '\n') {
        if (first < 0) first = cnt;
        if (cnt == first && cnt > 0) ++consistent;
        ++lines; cnt = 0;
      }
    }
    int score = consistent * 1000 + (first > 0 ? first : 0);
    if (c == ' ') score -= 500;  // space only if nothing else works
    if (score > best) { best = score; bsep = c; }
  }
  return bsep;
}

void* h2o_csv_parse(const char* buf, int64_t len, char sep, int header /*-1 guess, 0 no, 1 yes*/,
                    char quote, int nthreads) {
  Result* r = new Result();
  std::vector<int64_t> starts = find_records(buf, len, quote);
  // drop trailing empty records
  auto blank = [&](size_t k) {
    int64_t a = starts[k], b = (k + 1 < starts.size()) ? starts[k + 1] : len;
    for (int64_t i = a; i < b; ++i) if (buf[i] != '\n' && buf[i] != '\r' && buf[i] != ' ') return false;
    return true;
  };
  std::vector<int64_t> recs;
  recs.reserve(starts.size() + 1);
  for (size_t k = 0; k < starts.size(); ++k) {
    if (blank(k)) continue;
    int64_t a = starts[k];
    // comment lines
    if (buf[a] == '#') continue;
    recs.push_back(k);
  }
  auto rec_span = [&](int64_t k, int64_t& a, int64_t& b) {
    a = starts[k]; b = (k + 1 < (int64_t)starts.size()) ? starts[k + 1] : len;
  };
  std::vector<int64_t> co; std::vector<int32_t> cl; std::vector<uint8_t> cq;
  if (recs.empty()) { r->nrows = 0; r->ncols = 0; return r; }
  int64_t a, b;
  rec_span(recs[0], a, b);
  int nc = split_record(buf, a, b, sep, quote, co, cl, cq);
  std::vector<std::string> first;
  int first_text = 0, first_num = 0;
  for (int c = 0; c < nc; ++c) {
    first.emplace_back(buf + co[c], (size_t)cl[c]);
    double v;
    if (parse_number(buf + co[c], cl[c], &v)) ++first_num; else if (!is_na_token(buf + co[c], cl[c])) ++first_text;
  }
  bool has_header = header == 1;
  if (header < 0) {
    // header if first row is all text and the second row has numbers where the first has text
    bool second_num = false;
    if (recs.size() > 1) {
      rec_span(recs[1], a, b);
      std::vector<int64_t> co2; std::vector<int32_t> cl2; std::vector<uint8_t> cq2;
      int n2 = split_record(buf, a, b, sep, quote, co2, cl2, cq2);
      for (int c = 0; c < n2 && c < nc; ++c) { double v; if (parse_number(buf + co2[c], cl2[c], &v)) second_num = true; }
    }
    has_header = first_num == 0 && first_text > 0 && (second_num || recs.size() == 1);
    if (first_num == 0 && first_text == nc && recs.size() > 1 && !second_num) {
      // all-text file: header if first row values are unique identifiers
      has_header = true;
    }
  }
  int64_t row0 = has_header ? 1 : 0;
  r->ncols = nc;
  if (has_header) r->header = first;
  const int64_t nrows = (int64_t)recs.size() - row0;
  r->nrows = nrows;
  for (int c = 0; c < nc; ++c) {
    Col* col = new Col();
    col->num.assign((size_t)nrows, NAN);
    col->kind.assign((size_t)nrows, 0);
    col->off.assign((size_t)nrows, 0);
    col->len.assign((size_t)nrows, 0);
    r->cols.push_back(col);
  }
  int nt = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
  nt = std::max(1, std::min(nt, 64));
  if (nrows < 20000) nt = 1;
  std::vector<std::thread> th;
  // per-thread column tallies, summed after the join (the threads must not add into the shared Col counters)
  std::vector<std::vector<int64_t>> ttext((size_t)nt, std::vector<int64_t>(nc, 0)), tnum((size_t)nt, std::vector<int64_t>(nc, 0));
  for (int t = 0; t < nt; ++t) {
    th.emplace_back([&, t]() {
      std::vector<int64_t> lco; std::vector<int32_t> lcl; std::vector<uint8_t> lcq;
      const int64_t lo = nrows * t / nt, hi = nrows * (t + 1) / nt;
      std::vector<int64_t>& vtext = ttext[(size_t)t];
      std::vector<int64_t>& vnum = tnum[(size_t)t];
      for (int64_t r_ = lo; r_ < hi; ++r_) {
        int64_t ra, rb;
        rec_span(recs[r_ + row0], ra, rb);
        const int n = split_record(buf, ra, rb, sep, quote, lco, lcl, lcq);
        for (int c = 0; c < nc && c < n; ++c) {
          Col* col = r->cols[c];
          const char* s = buf + lco[c];
          const int l = lcl[c];
          col->off[r_] = lco[c];
          col->len[r_] = lcq[c] == 2 ? -l : l;  // negative length: contains escaped quotes
          double v;
          if (lcq[c] == 0 && is_na_token(s, l)) { col->kind[r_] = 0; }
          else if (parse_number(s, l, &v)) { col->num[r_] = v; col->kind[r_] = 1; ++vnum[c]; }
          else if (l == 0) { col->kind[r_] = 0; }
          else { col->kind[r_] = 2; ++vtext[c]; }
        }
      }
    });
  }
  for (auto& x : th) x.join();
  for (int t = 0; t < nt; ++t)
    for (int c = 0; c < nc; ++c) { r->cols[c]->n_text += ttext[(size_t)t][c]; r->cols[c]->n_num += tnum[(size_t)t][c]; }
  return r;
}

int64_t h2o_csv_nrows(void* h) { return ((Result*)h)->nrows; }
int h2o_csv_ncols(void* h) { return ((Result*)h)->ncols; }
int h2o_csv_has_header(void* h) { return ((Result*)h)->header.empty() ? 0 : 1; }
int64_t h2o_csv_count(void* h, int c, int kind) {
  Col* col = ((Result*)h)->cols[c];
  return kind == 1 ? col->n_num.load() : col->n_text.load();
}
int h2o_csv_header(void* h, int c, char* out, int cap) {
  Result* r = (Result*)h;
  if (c >= (int)r->header.size()) return -1;
  const std::string& s = r->header[c];
  int n = std::min<int>((int)s.size(), cap - 1);
  std::memcpy(out, s.data(), (size_t)n);
  out[n] = 0;
  return n;
}
int h2o_csv_get(void* h, int c, double* num, uint8_t* kind, int64_t* off, int32_t* len) {
  Result* r = (Result*)h;
  Col* col = r->cols[c];
  const size_t n = (size_t)r->nrows;
  if (n == 0) return 0;                 // (empty vectors: data() may be null, and memcpy from null is undefined)
  if (num) std::memcpy(num, col->num.data(), n * sizeof(double));
  if (kind) std::memcpy(kind, col->kind.data(), n);
  if (off) std::memcpy(off, col->off.data(), n * sizeof(int64_t));
  if (len) std::memcpy(len, col->len.data(), n * sizeof(int32_t));
  return 0;
}
void h2o_csv_free(void* h) { delete (Result*)h; }

// Build an enum domain for a text column: distinct strings (sorted) + per-row codes (-1 = NA).
// Numbers in a text column are kept as their literal token (H2O turns mixed columns into enums).
struct Domain { std::vector<std::string> levels; };
void* h2o_csv_domain(void* h, const char* buf, int c, int32_t* codes) {
  Result* r = (Result*)h;
  Col* col = r->cols[c];
  const int64_t n = r->nrows;
  std::vector<std::pair<std::string, int64_t>> items;
  items.reserve((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    if (col->kind[i] == 0) { codes[i] = -1; continue; }
    int32_t l = col->len[i];
    std::string s;
    if (l < 0) {  // unescape "" -> "
      l = -l;
      s.reserve((size_t)l);
      for (int32_t k = 0; k < l; ++k) { const char ch = buf[col->off[i] + k]; s.push_back(ch); if (ch == '"' && k + 1 < l && buf[col->off[i] + k + 1] == '"') ++k; }
    } else s.assign(buf + col->off[i], (size_t)l);
    items.emplace_back(std::move(s), i);
  }
  std::sort(items.begin(), items.end());
  Domain* d = new Domain();
  for (size_t k = 0; k < items.size(); ++k) {
    if (k == 0 || items[k].first != items[k - 1].first) d->levels.push_back(items[k].first);
    codes[items[k].second] = (int32_t)d->levels.size() - 1;
  }
  return d;
}
int h2o_domain_size(void* d) { return (int)((Domain*)d)->levels.size(); }
int h2o_domain_level(void* d, int k, char* out, int cap) {
  const std::string& s = ((Domain*)d)->levels[k];
  int n = std::min<int>((int)s.size(), cap - 1);
  std::memcpy(out, s.data(), (size_t)n);
  out[n] = 0;
  return (int)s.size();
}
void h2o_domain_free(void* d) { delete (Domain*)d; }

}  // extern "C"
