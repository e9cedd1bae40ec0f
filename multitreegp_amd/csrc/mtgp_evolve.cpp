// mtgp_evolve.cpp -- the reference's evolution step (genetic_operators/, gp.py:475-525) as a
// native host library, so a whole generation at BASELINE scale costs milliseconds next to the GPU
// evaluation.  Same operators, probabilities and array contract as the numpy restatement
// (multitreegp_amd/genetic_operators.py, the tested spec): a tree is float32 [N, 4] rows
// [f, a, b, value], empty rows packed low, root at row N-1, descending rows in preorder,
// a = k-1, b = k-1-|subtree(a)|.  Edits are done on the preorder node list and written back.
//
// Random numbers: xoshiro256** streams, one per (population, pair) derived from the seed, so the
// pairs of a population are independent and run on plain std::threads (contiguous blocks, no
// OpenMP runtime to spin beside torch's) with a result that does not depend on the thread count.  Runs are distributed like the reference's (JAX threefry keys split
// per operation), not draw for draw.
//
// References: initialization.py:9-164 (sample_tree), mutation.py:9-579, crossover.py:8-218,
// reproduction.py:8-176, genetic_programming.py:475-525.
#include <sched.h>
#include <stdint.h>
#include <string.h>
#include <xmmintrin.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <numeric>
#include <thread>
#include <vector>

#include "mtgp_host.h"

namespace {

// ---------------------------------------------------------------- random numbers
struct Rng {
  uint64_t s[4];
  static uint64_t splitmix(uint64_t& x) {
    uint64_t z = (x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  Rng(uint64_t seed, uint64_t a, uint64_t b) {
    uint64_t x = seed ^ (a * 0xd1342543de82ef95ull) ^ (b * 0x9e3779b97f4a7c15ull + 0x632be59bd9b4e019ull);
    for (int i = 0; i < 4; ++i) s[i] = splitmix(x);
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  double uniform() { return (double)(next() >> 11) * 0x1.0p-53; }
  int integer(int n) { return (int)((next() >> 32) * (uint64_t)n >> 32); }  // [0, n)
  double normal() {  // Marsaglia polar
    for (;;) {
      const double u = 2.0 * uniform() - 1.0, v = 2.0 * uniform() - 1.0, q = u * u + v * v;
      if (q > 0.0 && q < 1.0) return u * std::sqrt(-2.0 * std::log(q) / q);
    }
  }
  // index drawn with weights w[0..n) (not all zero)
  int choice(const double* w, int n) {
    double tot = 0.0;
    for (int i = 0; i < n; ++i) tot += w[i];
    double u = uniform() * tot;
    int last = 0;
    for (int i = 0; i < n; ++i) {
      if (w[i] <= 0.0) continue;
      last = i;
      if (u < w[i]) return i;
      u -= w[i];
    }
    return last;
  }
};

struct Node {
  int32_t f;
  float v;
};
typedef std::vector<Node> Nodes;

// Copy n floats of tree rows; non-temporal stores when the destination is 16-B aligned (the
// offspring array is written once and read by the next H2D copy: no read-for-ownership traffic,
// which at C5's 537 MB per generation is a third of the step's memory traffic).
inline void copy_rows(float* dst, const float* src, size_t n) {
  if (((uintptr_t)dst & 15u) != 0) {
    memcpy(dst, src, sizeof(float) * n);
    return;
  }
  size_t k = 0;
  for (; k + 4 <= n; k += 4) _mm_stream_ps(dst + k, _mm_loadu_ps(src + k));
  for (; k < n; ++k) dst[k] = src[k];
}

// ------------------------------------------------------------------ the library
struct Lib {
  const MtgpEvolveConfig* c;
  std::vector<double> op_p;
  std::vector<char> op_tab;  // op_tab[k]: k is an operator index (is_op as one lookup)
  void init(const MtgpEvolveConfig* cfg) {
    c = cfg;
    op_p.assign(cfg->op_prob, cfg->op_prob + cfg->n_ops);
    op_tab.assign(cfg->n_funcs > 0 ? cfg->n_funcs : 1, 0);
    for (int i = 0; i < cfg->n_ops; ++i)
      if (cfg->op_index[i] >= 0 && cfg->op_index[i] < cfg->n_funcs) op_tab[cfg->op_index[i]] = 1;
  }
  int arity(int f) const { return (f >= 0 && f < c->n_funcs) ? c->slots[f] : 0; }
  bool is_op(float f) const {  // f == (float)op_index[i] for some i (op indices are in [0, n_funcs))
    if (!(f >= 0.0f && f < (float)c->n_funcs)) return false;
    const int k = (int)f;
    return (float)k == f && op_tab[k];
  }
  bool is_var(float f) const { return f >= (float)c->var_start && f < (float)(c->var_start + c->n_vars); }
  bool is_leaf(float f) const { return f == 1.0f || is_var(f); }
};

// -------------------------------------------------------------- layout helpers
int find_end_idx(const float* t, int idx) {  // mutation.py:9-26
  int open = 1, k = idx;
  while (open > 0 && k >= 0) {
    open -= 1;
    open += (t[4 * k + 1] >= 0.0f) + (t[4 * k + 2] >= 0.0f);
    --k;
  }
  return k;
}

Nodes to_preorder(const float* t, int N) {
  Nodes out;
  for (int k = N - 1; k >= 0; --k) {
    const int f = (int)t[4 * k];
    if (f == 0) break;
    out.push_back({f, t[4 * k + 3]});
  }
  return out;
}

std::vector<int> subtree_sizes(const Nodes& n, const Lib& L) {
  std::vector<int> sz(n.size()), st;
  for (int i = (int)n.size() - 1; i >= 0; --i) {
    int s = 1;
    for (int a = 0; a < L.arity(n[i].f); ++a) {
      s += st.back();
      st.pop_back();
    }
    sz[i] = s;
    st.push_back(s);
  }
  return sz;
}

// preorder -> [N, 4]; false when the tree does not fit (the tree is left untouched)
bool from_preorder(const Nodes& n, const Lib& L, int N, float* t) {
  if ((int)n.size() > N || n.empty()) return false;
  const std::vector<int> sz = subtree_sizes(n, L);
  for (int k = 0; k < N; ++k) {
    t[4 * k + 0] = 0.0f;
    t[4 * k + 1] = -1.0f;
    t[4 * k + 2] = -1.0f;
    t[4 * k + 3] = 0.0f;
  }
  for (size_t i = 0; i < n.size(); ++i) {
    const int k = N - 1 - (int)i, ar = L.arity(n[i].f);
    t[4 * k + 0] = (float)n[i].f;
    t[4 * k + 1] = ar >= 1 ? (float)(k - 1) : -1.0f;
    t[4 * k + 2] = ar == 2 ? (float)(k - 1 - sz[i + 1]) : -1.0f;
    t[4 * k + 3] = n[i].f == 1 ? n[i].v : 0.0f;
  }
  return true;
}

// ---------------------------------------------------------------- the operators
struct Ops {
  Lib L;
  int N, depth;
  float sd;
  std::vector<int64_t> map_b_to_d;

  // initialization.py:9-124 for one tree: breadth-first draws, operators only while
  // open_slots < N - i - 1 and depth + 1 < depth_limit, leaf = coefficient w.p. 0.5 else an allowed
  // variable; the result in preorder (descending depth-first rows)
  Nodes sample_tree(Rng& g, int depth_limit, const float* var_mask) const {
    const int tree_size = (1 << depth) - 1, I = std::min(tree_size, 2 * N - 1);
    std::vector<int> f(I, 0);
    std::vector<float> coef(I, 0.0f);
    std::vector<double> vw(L.c->n_vars);
    for (int i = 0; i < L.c->n_vars; ++i) vw[i] = var_mask[i];
    int open = 1;
    for (int i = 0; i < I && open > 0; ++i) {
      const int d = 31 - __builtin_clz((unsigned)(i + 1));
      const float c = (float)(g.normal() * sd);
      int leaf = g.uniform() < 0.5 ? 1 : L.c->var_start + g.choice(vw.data(), L.c->n_vars);
      int index = leaf;
      if (open < N - i - 1 && d + 1 < depth_limit && g.uniform() < std::pow(0.7, d))
        index = L.c->op_index[g.choice(L.op_p.data(), L.c->n_ops)];
      if (i > 0) {
        const int pf = f[(i + (i % 2) - 2) / 2];
        if (!(L.arity(pf) + i % 2 > 1)) index = 0;
      }
      f[i] = index;
      coef[i] = index == 1 ? c : 0.0f;
      if (index != 0) open = std::max(0, open + L.arity(index) - 1);
    }
    Nodes out;
    std::vector<int> stack = {0};
    while (!stack.empty()) {  // preorder = first operand first
      const int i = stack.back();
      stack.pop_back();
      if (i >= I || f[i] == 0) continue;
      out.push_back({f[i], coef[i]});
      const int ar = L.arity(f[i]);
      if (ar >= 2) stack.push_back(2 * i + 2);
      if (ar >= 1) stack.push_back(2 * i + 1);
    }
    return out;
  }

  Node new_leaf(Rng& g, const float* var_mask) const {  // mutation.py:60, 188
    const float c = (float)(g.normal() * sd);
    if (g.uniform() < 0.5) return {1, c};
    std::vector<double> vw(L.c->n_vars);
    for (int i = 0; i < L.c->n_vars; ++i) vw[i] = var_mask[i];
    return {L.c->var_start + g.choice(vw.data(), L.c->n_vars), 0.0f};
  }
  int new_operator(Rng& g) const { return L.c->op_index[g.choice(L.op_p.data(), L.c->n_ops)]; }

  int choose_row(Rng& g, const std::vector<double>& w) const { return g.choice(w.data(), N); }
  std::vector<double> leaf_w(const float* t) const {
    std::vector<double> w(N);
    for (int k = 0; k < N; ++k) w[k] = L.is_leaf(t[4 * k]) ? 1.0 : 0.0;
    return w;
  }
  std::vector<double> op_w(const float* t, bool no_root) const {
    std::vector<double> w(N);
    for (int k = 0; k < N; ++k) w[k] = L.is_op(t[4 * k]) ? 1.0 : 0.0;
    if (no_root) w[N - 1] = 0.0;
    return w;
  }
  static bool any(const std::vector<double>& w) {
    for (double x : w)
      if (x > 0.0) return true;
    return false;
  }

  // replace the subtree rooted at `row` by `sub` (preorder); false if it does not fit
  bool replace(const float* t, int row, const Nodes& sub, float* out) const {
    const Nodes n = to_preorder(t, N);
    const int p = N - 1 - row;
    const int size = subtree_sizes(n, L)[p];
    Nodes m(n.begin(), n.begin() + p);
    m.insert(m.end(), sub.begin(), sub.end());
    m.insert(m.end(), n.begin() + p + size, n.end());
    return from_preorder(m, L, N, out);
  }
  Nodes subtree(const float* t, int row) const {
    const Nodes n = to_preorder(t, N);
    const int p = N - 1 - row;
    const int size = subtree_sizes(n, L)[p];
    return Nodes(n.begin() + p, n.begin() + p + size);
  }

  // -- the seven mutations (mutation.py:127-503); each writes `out`, false = unchanged
  bool add_subtree(const float* t, Rng& g, const float* vm, float* out) const {
    const std::vector<double> w = leaf_w(t);
    if (!any(w)) return false;
    const int row = choose_row(g, w);
    return replace(t, row, sample_tree(g, 2, vm), out);
  }
  bool mutate_leaf(const float* t, Rng& g, const float* vm, float* out) const {
    const std::vector<double> w = leaf_w(t);
    if (!any(w)) return false;
    for (int it = 0; it < kMaxRetries; ++it) {
      const int row = choose_row(g, w);
      const Node nl = new_leaf(g, vm);
      if (!(t[4 * row] == (float)nl.f && nl.f != 1)) {
        memcpy(out, t, sizeof(float) * 4 * N);
        out[4 * row] = (float)nl.f;
        out[4 * row + 3] = nl.f == 1 ? nl.v : 0.0f;
        return true;
      }
    }
    return false;
  }
  bool mutate_operator(const float* t, Rng& g, const float* vm, float* out) const {
    const std::vector<double> w = op_w(t, false);
    if (!any(w)) return false;
    int empty = 0;
    for (int k = 0; k < N; ++k) empty += t[4 * k] == 0.0f;
    int row = -1, op = 0;
    for (int it = 0; it < kMaxRetries; ++it) {
      const int r = choose_row(g, w);
      const int o = new_operator(g);
      const int size = r - find_end_idx(t, r);
      const int need = L.arity(o) == 2 ? 7 : 8;
      if (!(t[4 * r] == (float)o || empty + size < need)) {
        row = r;
        op = o;
        break;
      }
    }
    if (row < 0) return false;
    const int cur = L.arity((int)t[4 * row]), nw = L.arity(op);
    if (cur == nw) {
      memcpy(out, t, sizeof(float) * 4 * N);
      out[4 * row] = (float)op;
      return true;
    }
    Nodes sub = {{op, 0.0f}};
    if (nw == 1) {
      const Nodes s = sample_tree(g, 2, vm);
      sub.insert(sub.end(), s.begin(), s.end());
    } else {
      const Nodes s1 = sample_tree(g, 1, vm), s2 = sample_tree(g, 1, vm);
      sub.insert(sub.end(), s1.begin(), s1.end());
      sub.insert(sub.end(), s2.begin(), s2.end());
    }
    return replace(t, row, sub, out);
  }
  bool delete_operator(const float* t, Rng& g, const float* vm, float* out) const {
    const std::vector<double> w = op_w(t, true);
    if (!any(w)) return false;
    const int row = choose_row(g, w);
    return replace(t, row, Nodes{new_leaf(g, vm)}, out);
  }
  bool prepend_operator(const float* t, Rng& g, const float* vm, float* out) const {
    const int op = new_operator(g);
    const Nodes sub = sample_tree(g, 2, vm);
    const bool second = g.uniform() < 0.5;
    const Nodes old = to_preorder(t, N);
    Nodes n = {{op, 0.0f}};
    if (L.arity(op) == 2) {
      const Nodes& first = second ? sub : old;
      const Nodes& last = second ? old : sub;
      n.insert(n.end(), first.begin(), first.end());
      n.insert(n.end(), last.begin(), last.end());
    } else {
      n.insert(n.end(), old.begin(), old.end());
    }
    return from_preorder(n, L, N, out);
  }
  bool insert_operator(const float* t, Rng& g, const float* vm, float* out) const {
    const std::vector<double> w = op_w(t, true);
    if (!any(w)) return false;
    const int row = choose_row(g, w);
    const int op = new_operator(g);
    const Nodes sub = sample_tree(g, 2, vm);
    const bool second = g.uniform() < 0.5;
    const Nodes old = subtree(t, row);
    Nodes n = {{op, 0.0f}};
    if (L.arity(op) == 2) {
      const Nodes& first = second ? sub : old;
      const Nodes& last = second ? old : sub;
      n.insert(n.end(), first.begin(), first.end());
      n.insert(n.end(), last.begin(), last.end());
    } else {
      n.insert(n.end(), old.begin(), old.end());
    }
    return replace(t, row, n, out);
  }
  bool replace_tree(const float* t, Rng& g, const float* vm, float* out) const {
    (void)t;
    return from_preorder(sample_tree(g, depth, vm), L, N, out);
  }

  void mutate_tree(const float* t, Rng& g, const float* vm, float* out) const {  // get_mutations, mutation.py:523-539
    int empty = 0;
    for (int k = 0; k < N; ++k) empty += t[4 * k] == 0.0f;
    const int used = N - empty;
    double p[7] = {1, 1, 1, 1, 1, 1, 1};
    if (empty < 8) { const double q[7] = {0, 1, 1, 1, 0, 0, 1}; memcpy(p, q, sizeof p); }
    if (used <= 3) { const double q[7] = {1, 1, 1, 0, 1, 0, 1}; memcpy(p, q, sizeof p); }
    if (used == 1) { const double q[7] = {1, 1, 0, 0, 1, 0, 1}; memcpy(p, q, sizeof p); }
    bool ok = false;
    switch (g.choice(p, 7)) {
      case 0: ok = add_subtree(t, g, vm, out); break;
      case 1: ok = mutate_leaf(t, g, vm, out); break;
      case 2: ok = mutate_operator(t, g, vm, out); break;
      case 3: ok = delete_operator(t, g, vm, out); break;
      case 4: ok = prepend_operator(t, g, vm, out); break;
      case 5: ok = insert_operator(t, g, vm, out); break;
      default: ok = replace_tree(t, g, vm, out); break;
    }
    if (!ok) copy_rows(out, t, 4 * (size_t)N);
  }

  // -- crossover (crossover.py:60-192)
  // Crossover of one tree pair (the same draws and results as splicing the preorder lists through
  // subtree() / replace(), written without them: one scan per parent, then the two offspring rows
  // are written straight from the parents' rows; C5's 64 trees per candidate made the per-call
  // work the cost of a generation).
  void crossover(const float* t1, const float* t2, Rng& g, float* o1, float* o2) const {
    thread_local Scan x1, x2;
    scan(t1, x1);
    scan(t2, x2);
    auto unchanged = [&]() {
      copy_rows(o1, t1, 4 * (size_t)N);
      copy_rows(o2, t2, 4 * (size_t)N);
    };
    if (x1.c[N] == 0 || x2.c[N] == 0) return unchanged();
    for (int it = 0; it < kMaxRetries; ++it) {
      const int i1 = choose_prefix(g, x1.c), i2 = choose_prefix(g, x2.c);
      if (cx_invalid_e(t1, t2, i1, i2, x1.e, x2.e)) continue;
      const int n1 = N - x1.lo, n2 = N - x2.lo, s1 = x1.sz[i1], s2 = x2.sz[i2];
      // t1 with its subtree at i1 replaced by t2's at i2 (and the converse): n1 - s1 + s2 nodes
      if (n1 - s1 + s2 <= N && n2 - s2 + s1 <= N && n1 - s1 + s2 > 0 && n2 - s2 + s1 > 0) {
        splice_rows(t1, x1, i1, s1, t2, x2, i2, s2, o1);
        splice_rows(t2, x2, i2, s2, t1, x1, i1, s1, o2);
      } else {
        unchanged();
      }
      return;
    }
    unchanged();
  }
  // One pass over a parent's rows, low to high: the crossover row weights (crossover.py: 0 empty,
  // 2 operator, 1 leaf) as prefix sums c -- the weights are small integers, so Rng::choice's
  // running subtraction and a binary search over the prefix sums pick the same row for every draw
  // -- the empty-row count e cx_invalid_e needs, the lowest row lo of the preorder (rows N-1 .. lo,
  // as to_preorder reads them) and every row's subtree size from the arities (subtree_sizes on the
  // array itself: the operands of row k are the subtrees rooted at k-1 and just below it).
  struct Scan {
    std::vector<int> c, sz;
    int e, lo;
  };
  void scan(const float* t, Scan& x) const {
    x.c.resize(N + 1);
    x.sz.resize(N);
    int* c = x.c.data();
    int* sz = x.sz.data();
    const char* op = L.op_tab.data();
    const int* slots = L.c->slots;
    const int nf = L.c->n_funcs;
    int e = 0, lo = 0, acc = 0;
    c[0] = 0;
    for (int k = 0; k < N; ++k) {
      const float f = t[4 * k];
      const int fi = (int)f;
      const bool in = fi >= 0 && fi < nf;
      // Lib::is_op and Lib::arity with one range test
      const bool isop = in && f >= 0.0f && (float)fi == f && op[fi];
      const int ar = in ? slots[fi] : 0;
      e += f == 0.0f;
      lo = fi == 0 ? k + 1 : lo;
      acc += f == 0.0f ? 0 : (isop ? 2 : 1);
      c[k + 1] = acc;
      int s = 1;
      if (ar >= 1 && k >= 1) {
        const int sa = sz[k - 1], kb = k - 1 - sa;
        s += sa;
        if (ar >= 2 && kb >= 0) s += sz[kb];
      }
      sz[k] = s;
    }
    x.e = e;
    x.lo = lo;
  }
  // Write one crossover offspring straight from the parents' rows: `a`'s rows above ia, then `b`'s
  // subtree at ib (sb rows), then `a`'s rows below its subtree at ia (sa rows), each row
  // [f, k-1 | -1, k-1-|subtree(k-1)| | -1, value if coefficient] exactly as from_preorder
  // writes the spliced preorder list.  The subtree sizes of `a`'s rows above ia are a's own plus
  // (sb - sa) for the ancestors of ia (the rows whose subtree contains it).  `a` and `b` may be
  // the same tree (both tournaments picked one candidate).
  void splice_rows(const float* a, const Scan& xa, int ia, int sa, const float* b, const Scan& xb, int ib,
                   int sb, float* o) const {
    const int d = sb - sa, n = N - xa.lo + d;  // offspring nodes
    const int* za = xa.sz.data();
    const int* zb = xb.sz.data();
    const int kb = ia - sb, lo = N - n;  // the inserted subtree is rows ia .. kb+1
    auto size_at = [&](int k) {  // subtree size of output row k (any segment)
      if (k > ia) {
        const int s = za[k];
        return k - s + 1 <= ia ? s + d : s;  // an ancestor of the splice point
      }
      if (k > kb) return zb[ib - (ia - k)];
      return za[k + d];
    };
    const bool nt = ((uintptr_t)o & 15u) == 0;
    auto put = [&](int k, float f, float x, float y, float v) {
      if (nt) _mm_stream_ps(o + 4 * k, _mm_set_ps(v, y, x, f));
      else { o[4 * k] = f; o[4 * k + 1] = x; o[4 * k + 2] = y; o[4 * k + 3] = v; }
    };
    auto row = [&](int k, const float* src, int bsize) {  // bsize: |subtree(k-1)| in the offspring
      const int f = (int)src[0], ar = L.arity(f);
      put(k, (float)f, ar >= 1 ? (float)(k - 1) : -1.0f, ar == 2 ? (float)(k - 1 - bsize) : -1.0f,
          f == 1 ? src[3] : 0.0f);
    };
    for (int k = 0; k < lo; ++k) put(k, 0.0f, -1.0f, -1.0f, 0.0f);
    for (int k = lo; k <= kb; ++k) row(k, a + 4 * (k + d), k >= 1 ? za[k - 1 + d] : 0);
    for (int k = kb + 1; k <= ia; ++k) {
      const int r = ib - (ia - k);
      row(k, b + 4 * r, k - 1 > kb ? zb[r - 1] : size_at(k - 1));
    }
    for (int k = ia + 1; k < N; ++k) row(k, a + 4 * k, size_at(k - 1));
  }
  // Rng::choice over integer weights w[k] = c[k + 1] - c[k] (c non-decreasing, c[N] > 0): the same
  // uniform draw, and u - w[0] - ... - w[i-1] < w[i]  <=>  u < c[i + 1] exactly (integer sums)
  int choose_prefix(Rng& g, const std::vector<int>& c) const {
    const double u = g.uniform() * (double)c[N];
    int lo = 0, hi = N - 1;  // first i with c[i + 1] > u
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((double)c[mid + 1] > u) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  }
  // cx_invalid with the empty-row counts of both trees given
  bool cx_invalid_e(const float* t1, const float* t2, int i1, int i2, int e1, int e2) const {
    const int s1 = i1 - find_end_idx(t1, i1), s2 = i2 - find_end_idx(t2, i2);
    bool equal = false;
    if (s1 == s2 && (N - e1 > 1 || N - e2 > 1)) {
      equal = true;
      for (int k = 0; k < s1; ++k) {
        const float* a = t1 + 4 * (i1 - k);
        const float* b = t2 + 4 * (i2 - k);
        const bool same_leaf = a[3] == b[3] && a[0] == 1.0f;
        if (!((a[0] == b[0] && a[0] > 1.0f) || same_leaf)) {
          equal = false;
          break;
        }
      }
    }
    return e1 < s2 - s1 || e2 < s1 - s2 || equal;
  }

  static constexpr int kMaxRetries = 1000;
};

// mask of trees to change: Bernoulli(p) per tree, at least one (mutation.py:28-41)
std::vector<char> tree_mask(Rng& g, int T, double p) {
  std::vector<char> m(T);
  for (;;) {
    bool anyone = false;
    for (int t = 0; t < T; ++t) anyone |= (m[t] = g.uniform() < p);
    if (anyone) return m;
  }
}

// Threads: MTGP_HOST_THREADS, else OMP_NUM_THREADS (the CPU share a GPU pool grants the job), else
// the process's CPU affinity, at most 64.
long host_threads() {
  if (const char* e = std::getenv("MTGP_HOST_THREADS")) return std::max(1L, std::atol(e));
  if (const char* e = std::getenv("OMP_NUM_THREADS")) return std::max(1L, std::min(64L, std::atol(e)));
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) return std::max(1L, std::min(64L, (long)CPU_COUNT(&set)));
  return 8;
}

// body(k) for k in [0, n) on host_threads() threads in contiguous blocks; a thread only for every
// `grain` items
template <class F>
void parallel_for(long n, long grain, F body) {
  long want = host_threads();
  const long hw = std::max(1L, (long)std::thread::hardware_concurrency());
  const long nt = std::max(1L, std::min({want, hw, n / std::max(1L, grain)}));
  if (nt == 1) {
    for (long k = 0; k < n; ++k) body(k);
    return;
  }
  std::vector<std::thread> th;
  for (long t = 0; t < nt; ++t)
    th.emplace_back([=, &body]() {
      for (long k = n * t / nt; k < n * (t + 1) / nt; ++k) body(k);
    });
  for (auto& x : th) x.join();
}

}  // namespace

extern "C" int mtgp_host_abi_version(void) { return MTGP_HOST_ABI_VERSION; }

extern "C" int mtgp_evolve_populations(const float* pops, const float* fitness, int32_t num_pop, int32_t pop_size,
                                       int32_t T, int32_t N, const MtgpEvolveConfig* cfg, uint64_t seed, float* out) {
  if (!pops || !fitness || !cfg || !out || num_pop < 1 || pop_size < 1 || T < 1 || N < 1 || N > 4096) return -1;
  if (cfg->n_ops < 1 || cfg->n_vars < 1 || cfg->n_funcs < 2 || cfg->max_init_depth < 1 || cfg->max_init_depth > 30 ||
      cfg->tournament_size < 1 || cfg->elite_size < 0 || cfg->elite_size > pop_size)
    return -1;
  const size_t tsz = (size_t)4 * N, csz = tsz * T, psz = csz * pop_size;
  Ops ops;
  ops.L.init(cfg);
  ops.N = N;
  ops.depth = cfg->max_init_depth;
  ops.sd = cfg->coefficient_sd;
  // ring migration (reproduction.py:110-131, 160-167): population i receives the best of i - 1,
  // replacing its worst; the fitness handed to selection keeps the pre-migration order
  std::vector<float> mig;
  const float* cur = pops;
  if (num_pop > 1 && cfg->migration_period > 0 && (cfg->current_generation + 1) % cfg->migration_period == 0) {
    mig.resize(psz * num_pop);
    for (int i = 0; i < num_pop; ++i) {
      const int snd = (i + num_pop - 1) % num_pop;
      const float* rf = fitness + (size_t)i * pop_size;
      const float* sf = fitness + (size_t)snd * pop_size;
      std::vector<int> ro(pop_size), so(pop_size);
      std::iota(ro.begin(), ro.end(), 0);
      std::iota(so.begin(), so.end(), 0);
      std::stable_sort(ro.begin(), ro.end(), [&](int a, int b) { return -rf[a] < -rf[b]; });
      std::stable_sort(so.begin(), so.end(), [&](int a, int b) { return sf[a] < sf[b]; });
      for (int k = 0; k < pop_size; ++k) {
        const float* src = k < cfg->migration_size ? pops + (size_t)snd * psz + so[k] * csz
                                                   : pops + (size_t)i * psz + ro[k] * csz;
        memcpy(mig.data() + (size_t)i * psz + k * csz, src, sizeof(float) * csz);
      }
    }
    cur = mig.data();
  }
  const int E = cfg->elite_size, n_pairs = (pop_size - E) / 2;
  const int out_size = E + 2 * n_pairs;
  for (int i = 0; i < num_pop; ++i) {
    const float* P = cur + (size_t)i * psz;
    const float* F = fitness + (size_t)i * pop_size;
    float* O = out + (size_t)i * csz * out_size;
    std::vector<int> order(pop_size);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return F[a] < F[b]; });
    for (int e = 0; e < E; ++e) memcpy(O + (size_t)e * csz, P + (size_t)order[e] * csz, sizeof(float) * csz);
    const double* tp = cfg->tournament_prob + (size_t)i * cfg->tournament_size;
    const double* rp = cfg->reproduction_type_prob + (size_t)i * 3;
    const double repro = cfg->reproduction_prob[i];
    // a thread per >= 64K tree rows of offspring (C5: 8 pairs, C3: 342 pairs)
    parallel_for(n_pairs, std::max(1L, 65536L / ((long)T * N)), [&](long k) {
      Rng g(seed, (uint64_t)i + 1, (uint64_t)k + 1);
      auto tournament = [&]() {  // reproduction.py:29-49
        thread_local std::vector<int> idx;
        idx.resize(cfg->tournament_size);
        for (int j = 0; j < cfg->tournament_size; ++j) idx[j] = g.integer(pop_size);
        std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return F[a] < F[b]; });
        return idx[g.choice(tp, cfg->tournament_size)];
      };
      const float* p1 = P + (size_t)tournament() * csz;
      const float* p2 = P + (size_t)tournament() * csz;
      float* c1 = O + (size_t)(E + k) * csz;
      float* c2 = O + (size_t)(E + n_pairs + k) * csz;
      const int type = g.choice(rp, 3);
      if (type == 0) {  // crossover_trees (crossover.py:194-218)
        const std::vector<char> m = tree_mask(g, T, repro);
        for (int t = 0; t < T; ++t) {
          if (m[t]) ops.crossover(p1 + t * tsz, p2 + t * tsz, g, c1 + t * tsz, c2 + t * tsz);
          else {
            copy_rows(c1 + t * tsz, p1 + t * tsz, tsz);
            copy_rows(c2 + t * tsz, p2 + t * tsz, tsz);
          }
        }
      } else if (type == 1) {  // mutate_pair (gp.py:499-511, mutation.py:555-577)
        for (int side = 0; side < 2; ++side) {
          const float* par = side ? p2 : p1;
          float* ch = side ? c2 : c1;
          const std::vector<char> m = tree_mask(g, T, repro);
          for (int t = 0; t < T; ++t) {
            if (m[t]) ops.mutate_tree(par + t * tsz, g, cfg->var_mask + (size_t)t * cfg->n_vars, ch + t * tsz);
            else copy_rows(ch + t * tsz, par + t * tsz, tsz);
          }
        }
      } else {  // sample_pair (gp.py:513-525): two fresh candidates
        for (int side = 0; side < 2; ++side) {
          float* ch = side ? c2 : c1;
          for (int t = 0; t < T; ++t)
            from_preorder(ops.sample_tree(g, ops.depth, cfg->var_mask + (size_t)t * cfg->n_vars), ops.L, N,
                          ch + t * tsz);
        }
      }
      _mm_sfence();  // the non-temporal row stores are visible before the threads join
    });
  }
  return out_size;
}

// one fresh tree per (population member, tree) -- initialize_population (gp.py:298-308)
extern "C" int mtgp_sample_population(int32_t num_pop, int32_t pop_size, int32_t T, int32_t N,
                                      const MtgpEvolveConfig* cfg, uint64_t seed, float* out) {
  if (!cfg || !out || num_pop < 1 || pop_size < 1 || T < 1 || N < 1 || N > 4096) return -1;
  Ops ops;
  ops.L.init(cfg);
  ops.N = N;
  ops.depth = cfg->max_init_depth;
  ops.sd = cfg->coefficient_sd;
  const long B = (long)num_pop * pop_size;
  parallel_for(B, 256, [&](long b) {
    Rng g(seed, 0x5a4d5045ull, (uint64_t)b + 1);
    for (int t = 0; t < T; ++t)
      from_preorder(ops.sample_tree(g, ops.depth, cfg->var_mask + (size_t)t * cfg->n_vars), ops.L, N,
                    out + ((size_t)b * T + t) * 4 * N);
  });
  return 0;
}
