#include <cstdio>
#include <cstdint>
#include <string>
extern "C" {
void* h2o_csv_parse(const char* buf, int64_t len, char sep, int header, char quote, int nthreads);
int64_t h2o_csv_nrows(void* h);
int64_t h2o_csv_count(void* h, int c, int kind);
void h2o_csv_free(void* h);
}
int main() {
  std::string s = "a,b,c\n";
  for (int i = 0; i < 60000; ++i) s += std::to_string(i) + "," + (i % 7 ? "x" : "NA") + "," + std::to_string(i * 0.5) + "\n";
  void* h = h2o_csv_parse(s.data(), (int64_t)s.size(), ',', 1, '"', 8);
  std::printf("rows %lld text1 %lld num0 %lld\n", (long long)h2o_csv_nrows(h), (long long)h2o_csv_count(h, 1, 2),
              (long long)h2o_csv_count(h, 0, 1));
  h2o_csv_free(h);
  return 0;
}
