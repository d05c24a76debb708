// Host stress test for the native batch loader under ThreadSanitizer / ASan+UBSan:
//   g++ -O1 -g -fsanitize=thread -pthread loader_stress.cpp ../../bigdl-1_amd/bigdl/runtime/csrc/batch_loader.cpp
// Pulls several epochs with 6 workers and 3 slots, checks every epoch is a permutation.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" {
void* bigdl_loader_create(const uint8_t*, const float*, long long, int, int, int, int, int, int, int, int, int, int,
                          const float*, const float*, int, int, int, int, unsigned long long, int, int, void**,
                          float**);
int bigdl_loader_next(void*, int*, long long*);
void bigdl_loader_release(void*, int);
void bigdl_loader_destroy(void*);
}

int main() {
  const int n = 97, h = 9, w = 7, c = 3, B = 8, K = 3;
  std::vector<uint8_t> img((size_t)n * h * w * c);
  for (size_t i = 0; i < img.size(); ++i) img[i] = (uint8_t)(i * 31);
  std::vector<float> lab(n);
  for (int i = 0; i < n; ++i) lab[i] = (float)i;
  std::vector<std::vector<float>> xs(K, std::vector<float>((size_t)B * c * 7 * 5)), ys(K, std::vector<float>(B));
  void* xp[K];
  float* yp[K];
  for (int k = 0; k < K; ++k) { xp[k] = xs[k].data(); yp[k] = ys[k].data(); }
  void* L = bigdl_loader_create(img.data(), lab.data(), n, h, w, c, 1, B, 7, 5, 1, 1, 1, nullptr, nullptr, 0, 0, 1, 1,
                                42, 6, K, xp, yp);
  if (!L) return 2;
  const int nb = n / B;
  for (int e = 0; e < 4; ++e) {
    std::vector<int> seen(n, 0);
    for (int b = 0; b < nb; ++b) {
      int rows = 0;
      long long bi = 0;
      const int s = bigdl_loader_next(L, &rows, &bi);
      if (bi != (long long)e * nb + b || rows != B) return 3;
      for (int r = 0; r < rows; ++r) seen[(int)ys[s][r]]++;
      bigdl_loader_release(L, s);
    }
    int dup = 0;
    for (int i = 0; i < n; ++i) dup += seen[i] > 1;
    if (dup) return 4;
  }
  bigdl_loader_destroy(L);
  std::printf("loader stress ok\n");
  return 0;
}
