// click_log.cpp — host-side builders of the DIN and triplet training rows over
// a typed CSR click log (typed click logs).
//
// The reference builds its rows in Python loops over {uid: [article ids]}
// dicts (DIN.py:66-76, embedding_generate.py:25-39), drawing each negative with
// `random.choice(article_ids)` until it is not in the user's clicks.  To give
// the SAME rows (a sample-exact drop-in, given the same `random` state) these
// builders replay CPython's Mersenne Twister and its `choice`:
//   choice(seq)     = seq[_randbelow(len(seq))]                  (random.py, 3.10)
//   _randbelow(n)   = k = n.bit_length(); r = getrandbits(k) until r < n
//   getrandbits(k)  = genrand_uint32() >> (32 - k)               (k <= 32)
// on the state tuple random.getstate()[1] (624 words + position), which the
// caller passes in and receives back advanced, so `random` continues exactly
// as if the reference loop had run.  The draws are inherently serial; the
// per-user membership test is a binary search over the user's sorted clicks
// instead of the reference's list scan.
//
// Host memory only (no HIP): the rows are built once per epoch setup and then
// copied to HBM, where the DIN kernels gather the embeddings (nrk_din_batch).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/nrk.h"
#include "nrk_common.h"

namespace {

// CPython's MT19937 (Modules/_randommodule.c: genrand_uint32), restated.
struct PyMT {
  static constexpr int N = 624, M = 397;
  uint32_t mt[N];
  int index;

  void load(const uint32_t* st) {
    memcpy(mt, st, sizeof(mt));
    index = (int)st[N];
  }
  void store(uint32_t* st) const {
    memcpy(st, mt, sizeof(mt));
    st[N] = (uint32_t)index;
  }
  void twist() {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    int kk = 0;
    uint32_t y;
    for (; kk < N - M; kk++) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + M] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < N - 1; kk++) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + (M - N)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (mt[N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[N - 1] = mt[M - 1] ^ (y >> 1) ^ mag01[y & 1u];
    index = 0;
  }
  uint32_t next() {
    if (index >= N) twist();
    uint32_t y = mt[index++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  // random.choice over a sequence of n (1 <= n < 2^32) elements: the index drawn
  uint32_t below(uint32_t n, int k) {
    uint32_t r;
    do {
      r = next() >> (32 - k);
    } while (r >= n);
    return r;
  }
};

int bit_length(uint64_t n) {
  int k = 0;
  while (n) {
    k++;
    n >>= 1;
  }
  return k;
}

// common argument checks; fills `sorted` per user lazily in the callers
int check_log(const int64_t* click_off, int64_t n_users, const int32_t* click_rows, int64_t n_items,
              const uint32_t* rng_state, const char* what) {
  if (n_users < 0 || !click_off || !rng_state) return nrk::fail(NRK_EINVAL, "%s: null pointer or n_users < 0", what);
  if (click_off[0] != 0) return nrk::fail(NRK_EINVAL, "%s: click_off[0] must be 0", what);
  for (int64_t u = 0; u < n_users; u++)
    if (click_off[u + 1] < click_off[u]) return nrk::fail(NRK_EINVAL, "%s: click_off not non-decreasing at %lld", what,
                                                          (long long)u);
  const int64_t nnz = click_off[n_users];
  if (nnz > 0 && !click_rows) return nrk::fail(NRK_EINVAL, "%s: click_rows is null", what);
  if (n_items < 0 || n_items >= (1ll << 32)) return nrk::fail(NRK_EINVAL, "%s: n_items out of range", what);
  for (int64_t j = 0; j < nnz; j++)
    if (click_rows[j] < 0 || click_rows[j] >= n_items)
      return nrk::fail(NRK_EINVAL, "%s: click row %d at %lld outside [0, %lld)", what, click_rows[j], (long long)j,
                       (long long)n_items);
  if (rng_state[PyMT::N] > (uint32_t)PyMT::N) return nrk::fail(NRK_EINVAL, "%s: bad Mersenne Twister position", what);
  return NRK_OK;
}

// sorted distinct clicks of one user (the membership set); returns false when
// they cover every item (the reference's rejection loop would never end)
bool user_set(const int32_t* rows, int64_t n, int64_t n_items, std::vector<int32_t>& s) {
  s.assign(rows, rows + n);
  std::sort(s.begin(), s.end());
  s.erase(std::unique(s.begin(), s.end()), s.end());
  return (int64_t)s.size() < n_items;
}

}  // namespace

extern "C" int nrk_train_samples(const int64_t* click_off, int64_t n_users, const int32_t* click_rows,
                                 int64_t n_items, int32_t max_history, uint32_t* rng_state, int64_t n_samples,
                                 int32_t* user_idx, int32_t* target_rows, float* labels, int32_t* hist_rows) {
  const char* what = "nrk_train_samples";
  int rc = check_log(click_off, n_users, click_rows, n_items, rng_state, what);
  if (rc) return rc;
  if (max_history < 1) return nrk::fail(NRK_EINVAL, "%s: max_history must be >= 1", what);
  int64_t need = 0;
  for (int64_t u = 0; u < n_users; u++) {
    const int64_t n = click_off[u + 1] - click_off[u];
    if (n > 1) need += 2 * (n - 1);
  }
  if (n_samples != need)
    return nrk::fail(NRK_EINVAL, "%s: n_samples = %lld, the log yields %lld", what, (long long)n_samples,
                     (long long)need);
  if (need > 0 && (!user_idx || !target_rows || !labels))
    return nrk::fail(NRK_EINVAL, "%s: null output pointer", what);
  if (need > 0 && n_items == 0) return nrk::fail(NRK_EINVAL, "%s: cannot choose from an empty sequence", what);

  PyMT mt;
  mt.load(rng_state);
  const uint32_t n = (uint32_t)n_items;
  const int k = bit_length(n);
  std::vector<int32_t> set;
  int64_t j = 0;
  for (int64_t u = 0; u < n_users; u++) {
    const int64_t s = click_off[u], len = click_off[u + 1] - s;
    if (len < 2) continue;  // range(1, len(clicks)) is empty
    const int32_t* c = click_rows + s;
    if (!user_set(c, len, n_items, set)) {
      mt.store(rng_state);
      return nrk::fail(NRK_EINVAL, "%s: user %lld clicked every item (no negative exists)", what, (long long)u);
    }
    for (int64_t i = 1; i < len; i++) {
      // DIN.py:72-76: history = clicks[:i][-L:], positive then negative
      const int64_t h0 = i > max_history ? i - max_history : 0;
      uint32_t neg;
      do {
        neg = mt.below(n, k);
      } while (std::binary_search(set.begin(), set.end(), (int32_t)neg));
      for (int half = 0; half < 2; half++, j++) {
        user_idx[j] = (int32_t)u;
        target_rows[j] = half == 0 ? c[i] : (int32_t)neg;
        labels[j] = half == 0 ? 1.0f : 0.0f;
        if (hist_rows) {
          int32_t* h = hist_rows + j * (int64_t)max_history;
          const int64_t hl = i - h0;
          for (int64_t t = 0; t < hl; t++) h[t] = c[h0 + t];
          for (int64_t t = hl; t < max_history; t++) h[t] = -1;
        }
      }
    }
  }
  mt.store(rng_state);
  return NRK_OK;
}

extern "C" int nrk_triplet_samples(const int64_t* click_off, int64_t n_users, const int32_t* click_rows,
                                   int64_t n_items, uint32_t* rng_state, int64_t n_triplets, int32_t* triplets) {
  const char* what = "nrk_triplet_samples";
  int rc = check_log(click_off, n_users, click_rows, n_items, rng_state, what);
  if (rc) return rc;
  int64_t need = 0;
  for (int64_t u = 0; u < n_users; u++) {
    const int64_t n = click_off[u + 1] - click_off[u];
    if (n >= 2) need += n * (n - 1) / 2;
  }
  if (n_triplets != need)
    return nrk::fail(NRK_EINVAL, "%s: n_triplets = %lld, the log yields %lld", what, (long long)n_triplets,
                     (long long)need);
  if (need > 0 && !triplets) return nrk::fail(NRK_EINVAL, "%s: null output pointer", what);
  if (need > 0 && n_items == 0) return nrk::fail(NRK_EINVAL, "%s: cannot choose from an empty sequence", what);

  PyMT mt;
  mt.load(rng_state);
  const uint32_t n = (uint32_t)n_items;
  const int k = bit_length(n);
  std::vector<int32_t> set;
  int64_t j = 0;
  for (int64_t u = 0; u < n_users; u++) {
    const int64_t s = click_off[u], len = click_off[u + 1] - s;
    if (len < 2) continue;  // embedding_generate.py:31
    const int32_t* c = click_rows + s;
    if (!user_set(c, len, n_items, set)) {
      mt.store(rng_state);
      return nrk::fail(NRK_EINVAL, "%s: user %lld clicked every item (no negative exists)", what, (long long)u);
    }
    for (int64_t a = 0; a + 1 < len; a++)
      for (int64_t p = a + 1; p < len; p++, j++) {  // embedding_generate.py:32-39
        uint32_t neg;
        do {
          neg = mt.below(n, k);
        } while (std::binary_search(set.begin(), set.end(), (int32_t)neg));
        triplets[3 * j + 0] = c[a];
        triplets[3 * j + 1] = c[p];
        triplets[3 * j + 2] = (int32_t)neg;
      }
  }
  mt.store(rng_state);
  return NRK_OK;
}
