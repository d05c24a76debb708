// Native multi-threaded minibatch assembler (the reference's MTLabeledBGRImgToBatch /
// MTImageFeatureToBatch: DL/dataset/image/MTLabeledBGRImgToBatch.scala, DL/transform/vision/image/
// MTImageFeatureToBatch.scala — worker threads crop / flip / normalise samples into a batch).
//
// Input: an in-memory uint8 image array [N][H][W][C] (HWC, any channel order) + float labels.
// Output: batches written by T worker threads straight into K caller-owned (pinned) slot buffers,
// as fp32 or bf16 in NCHW or NHWC, ready for an asynchronous H2D copy.  Per sample: optional zero
// padding + random crop (train) or center crop (eval), optional random horizontal flip, then
// (pixel - mean[c]) / std[c].  Every batch index b is a pure function of (seed, b): epoch b / nb
// uses its own shuffled permutation (Fisher-Yates on mt19937_64(seed + epoch)), and sample i of
// batch b draws its crop/flip from mt19937_64(seed ^ hash(b, i)) — results do not depend on the
// thread count or timing.  The iterator is infinite (train mode of CachedDistriDataSet).
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#define EXPORT extern "C" __attribute__((visibility("default")))

namespace {

inline uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);                                           // round to nearest even
  return (uint16_t)(u >> 16);
}

inline uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

enum SlotState { FREE = 0, FILLING = 1, READY = 2 };

struct Loader {
  const uint8_t* data;
  const float* labels;
  int64_t n;
  int h, w, c, label_dim;
  int batch, ch, cw, pad, flip, train, bf16, nhwc, shuffle, drop_last;
  std::vector<float> mean, inv_std;
  uint64_t seed;
  int64_t nb;  // batches per epoch
  std::vector<void*> slots_x;
  std::vector<float*> slots_y;
  std::vector<int> state;
  std::vector<int64_t> slot_batch;
  std::vector<int> slot_rows;
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<int64_t> next_claim{0};
  int64_t next_serve = 0;
  bool stop = false;
  std::vector<std::thread> workers;
  // permutations cached per epoch (two live epochs at most)
  std::mutex perm_mu;
  int64_t perm_epoch[2] = {-1, -1};
  std::vector<int64_t> perm[2];

  const std::vector<int64_t>& permutation(int64_t epoch) {
    std::lock_guard<std::mutex> g(perm_mu);
    for (int i = 0; i < 2; ++i)
      if (perm_epoch[i] == epoch) return perm[i];
    const int k = (int)(epoch & 1);
    perm[k].resize(n);
    for (int64_t i = 0; i < n; ++i) perm[k][i] = i;
    if (shuffle) {
      std::mt19937_64 g64(seed + 0x9E3779B97F4A7C15ULL * (uint64_t)(epoch + 1));
      for (int64_t i = n - 1; i > 0; --i) {
        std::uniform_int_distribution<int64_t> d(0, i);
        std::swap(perm[k][i], perm[k][d(g64)]);
      }
    }
    perm_epoch[k] = epoch;
    return perm[k];
  }

  void fill(int slot, int64_t b) {
    const int64_t epoch = b / nb, off = (b % nb) * batch;
    const std::vector<int64_t>& p = permutation(epoch);
    const int rows = (int)std::min<int64_t>(batch, n - off);
    const size_t plane = (size_t)ch * cw;
    for (int r = 0; r < rows; ++r) {
      const int64_t idx = p[off + r];
      const uint8_t* img = data + (size_t)idx * h * w * c;
      std::mt19937_64 g64(mix(seed ^ mix((uint64_t)b * 1315423911ULL + (uint64_t)r)));
      int oy, ox;  // crop origin in padded coordinates
      if (train) {
        oy = (int)(g64() % (uint64_t)(h + 2 * pad - ch + 1));
        ox = (int)(g64() % (uint64_t)(w + 2 * pad - cw + 1));
      } else {
        oy = (h + 2 * pad - ch) / 2;
        ox = (w + 2 * pad - cw) / 2;
      }
      const bool fl = flip && train && (g64() & 1);
      for (int y = 0; y < ch; ++y) {
        const int sy = oy + y - pad;
        for (int x = 0; x < cw; ++x) {
          const int xx = fl ? (cw - 1 - x) : x;
          const int sx = ox + xx - pad;
          const bool in = sy >= 0 && sy < h && sx >= 0 && sx < w;
          const uint8_t* px = in ? img + ((size_t)sy * w + sx) * c : nullptr;
          for (int k = 0; k < c; ++k) {
            const float v = ((in ? (float)px[k] : 0.f) - mean[k]) * inv_std[k];
            const size_t o = nhwc ? (((size_t)r * ch + y) * cw + x) * c + k
                                  : ((size_t)r * c + k) * plane + (size_t)y * cw + x;
            if (bf16)
              ((uint16_t*)slots_x[slot])[o] = f2bf(v);
            else
              ((float*)slots_x[slot])[o] = v;
          }
        }
      }
      if (labels)
        std::memcpy(slots_y[slot] + (size_t)r * label_dim, labels + (size_t)idx * label_dim,
                    sizeof(float) * label_dim);
    }
    slot_rows[slot] = rows;
  }

  void worker() {
    const int K = (int)slots_x.size();
    for (;;) {
      const int64_t b = next_claim.fetch_add(1);
      const int slot = (int)(b % K);
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || (state[slot] == FREE && b - next_serve < K); });
        if (stop) return;
        state[slot] = FILLING;
        slot_batch[slot] = b;
      }
      fill(slot, b);
      {
        std::lock_guard<std::mutex> lk(mu);
        state[slot] = READY;
      }
      cv.notify_all();
    }
  }
};

}  // namespace

// Returns an opaque handle or null on invalid arguments.  `slots_x[K]` / `slots_y[K]` are the
// caller's batch buffers (batch·C·crop_h·crop_w elements of fp32/bf16, batch·label_dim floats).
EXPORT void* bigdl_loader_create(const uint8_t* data, const float* labels, long long n, int h, int w, int c,
                                 int label_dim, int batch, int crop_h, int crop_w, int pad, int flip, int train,
                                 const float* mean, const float* std, int bf16, int nhwc, int shuffle,
                                 int drop_last, unsigned long long seed, int threads, int k, void** slots_x,
                                 float** slots_y) {
  if (!data || n <= 0 || h <= 0 || w <= 0 || c <= 0 || batch <= 0 || crop_h <= 0 || crop_w <= 0 || pad < 0 ||
      crop_h > h + 2 * pad || crop_w > w + 2 * pad || threads <= 0 || k < 1 || (labels && label_dim <= 0))
    return nullptr;
  if (drop_last && n < batch) return nullptr;
  Loader* L = new Loader();
  L->data = data;
  L->labels = labels;
  L->n = n;
  L->h = h; L->w = w; L->c = c; L->label_dim = label_dim;
  L->batch = batch; L->ch = crop_h; L->cw = crop_w; L->pad = pad; L->flip = flip; L->train = train;
  L->bf16 = bf16; L->nhwc = nhwc; L->shuffle = shuffle; L->drop_last = drop_last;
  L->seed = seed;
  L->nb = drop_last ? n / batch : (n + batch - 1) / batch;
  for (int i = 0; i < c; ++i) {
    L->mean.push_back(mean ? mean[i] : 0.f);
    L->inv_std.push_back(std ? 1.f / std[i] : 1.f);
  }
  for (int i = 0; i < k; ++i) {
    L->slots_x.push_back(slots_x[i]);
    L->slots_y.push_back(slots_y ? slots_y[i] : nullptr);
  }
  L->state.assign(k, FREE);
  L->slot_batch.assign(k, -1);
  L->slot_rows.assign(k, 0);
  for (int t = 0; t < threads; ++t) L->workers.emplace_back([L] { L->worker(); });
  return L;
}

// Blocks until the next batch (in order) is ready; returns its slot, and its row count / global
// batch index through the out-params.  The slot stays owned by the caller until released.
EXPORT int bigdl_loader_next(void* h, int* rows, long long* batch_index) {
  Loader* L = (Loader*)h;
  const int K = (int)L->slots_x.size();
  std::unique_lock<std::mutex> lk(L->mu);
  const int64_t b = L->next_serve;
  const int slot = (int)(b % K);
  L->cv.wait(lk, [&] { return L->state[slot] == READY && L->slot_batch[slot] == b; });
  L->next_serve++;
  if (rows) *rows = L->slot_rows[slot];
  if (batch_index) *batch_index = b;
  return slot;
}

EXPORT void bigdl_loader_release(void* h, int slot) {
  Loader* L = (Loader*)h;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->state[slot] = FREE;
  }
  L->cv.notify_all();
}

EXPORT long long bigdl_loader_batches_per_epoch(void* h) { return ((Loader*)h)->nb; }

EXPORT void bigdl_loader_destroy(void* h) {
  Loader* L = (Loader*)h;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->stop = true;
  }
  L->cv.notify_all();
  for (auto& t : L->workers) t.join();
  delete L;
}
