#include <cstdio>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>
extern "C" {
void* h2o_csv_parse(const char* buf, int64_t len, char sep, int header, char quote, int nthreads);
int64_t h2o_csv_nrows(void* h);
int h2o_csv_ncols(void* h);
int h2o_csv_get(void* h, int c, double* num, uint8_t* kind, int64_t* off, int32_t* len);
void h2o_csv_free(void* h);
char h2o_csv_guess_sep(const char* buf, int64_t len);
}
int main() {
  std::vector<std::string> cases = {"", "\n", "a", "a,b\n1,2", "a,b\n\"x,y\",2\n\"q\"\"q\",3\n", "a\n\"unterminated\n",
                                    "a,b,c\n1\n1,2,3,4,5\n", ",,,\n,,,\n", "x;y\n1;2\n", "\"\"\n\"\"\n", "a\r\n1\r\n2\r\n"};
  std::string big = "h1,h2\n";
  for (int i = 0; i < 30000; ++i) big += (i % 3 ? "\"a,\"\"b\"" : std::to_string(i)) + std::string(",") + std::to_string(i) + "\n";
  cases.push_back(big);
  for (auto& c : cases) {
    std::vector<char> buf(c.begin(), c.end());            // exact-size heap buffer: overreads are reported
    const char* p = buf.empty() ? "" : buf.data();
    char sep = h2o_csv_guess_sep(p, (int64_t)buf.size());
    void* h = h2o_csv_parse(p, (int64_t)buf.size(), sep ? sep : ',', -1, '"', 4);
    if (!h) continue;
    const int64_t n = h2o_csv_nrows(h);
    for (int col = 0; col < h2o_csv_ncols(h); ++col) {
      std::vector<double> num((size_t)n + 1); std::vector<uint8_t> kind((size_t)n + 1);
      std::vector<int64_t> off((size_t)n + 1); std::vector<int32_t> len((size_t)n + 1);
      h2o_csv_get(h, col, num.data(), kind.data(), off.data(), len.data());
    }
    std::printf("case %zu bytes -> %lld rows %d cols\n", c.size(), (long long)n, h2o_csv_ncols(h));
    h2o_csv_free(h);
  }
  return 0;
}
