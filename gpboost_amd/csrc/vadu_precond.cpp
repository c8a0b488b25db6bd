// VaduPrecond implementation: host planning of the three-part VADU solves and their launch
// sequence (vadu_precond.h explains the split).
#include "vadu_precond.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>

namespace gpb_amd {

VaduPrecond::~VaduPrecond() { DropGraphs(); }

void VaduPrecond::DropGraphs() {
  if (graphs_.empty()) return;
  // A replay may still be in flight (Scratch grows S_ between two applications of one PCG, on
  // possibly different streams): its exec, kernel-argument pool and scratch must outlive it, and a
  // kernel tracer reads the dispatches' arguments after they ran. Rare (a new width, a new dw).
  (void)hipDeviceSynchronize();
  for (GraphEntry& g : graphs_) (void)hipGraphExecDestroy(g.exec);
  graphs_.clear();
}

int VaduPrecond::launches() const {
  int c = tail_persist_ ? 2 : tail_levels_bt() + tail_levels_lower();
  if (K_ > 0) ++c;                          // tail -> head partial
  if (K_ > K0_) c += 2;                     // the two segment solves
  if (K0_ > 0) c += 2 + (K_ > K0_ ? 2 : 0); // two dense products (+ the two head-1 <-> head-0 partials)
  return c;
}

namespace {
// Host side of one solve's merged tail (latent_kernels.h, MergedSolve): rows in level order,
// g levels per merged level; deps(i, f) calls f(dependency row, value slot) for row i's entries
// in order; in_tail(j) says whether row j is solved in this tail.
struct MergeHost {
  std::vector<int> rows, eoff{0}, xoff, eidx;
  std::vector<int> opoff{0}, op_a, op_slot, op_map, map;
  std::vector<int> lptr{0};
  std::vector<int> offpos, offptr;
};

// Levels are merged greedily in order: a merged level takes the next level while its entries
// (fill included) stay within `budget` and it spans at most gmax levels. Fat levels (throughput-
// bound already) stay alone; runs of thin ones (launch-bound) are merged deeply.
template <class Deps, class InTail>
void build_merged(int n, long budget, int gmax, const std::vector<std::vector<int>>& levels, Deps deps,
                  InTail in_tail, MergeHost& h) {
  const int L = (int)levels.size();
  std::vector<int> pos_of(n, -1), grp(n, -1);
  int P = 0;
  for (int l = 0; l < L; ++l)
    for (int r : levels[l]) pos_of[r] = P++;
  std::vector<std::vector<int>> by_off(std::max(1, gmax));
  std::vector<int> keypos(2 * (size_t)n, -1);   // list position of a key (X entry: j; IN entry: n + j)
  std::vector<int> keys, lmap, perm;
  struct Op { int a, slot, map; };
  std::vector<Op> ops;
  int G = 0, l0 = 0;   // current merged level and its first level
  long gent = 0;       // entries of the current merged level
  for (int l = 0; l < L; ++l) {
    for (int attempt = 0; attempt < 2; ++attempt) {
      const size_t c_rows = h.rows.size(), c_eidx = h.eidx.size(), c_ops = h.op_a.size(), c_map = h.map.size();
      for (int r : levels[l]) grp[r] = G;
      for (int i : levels[l]) {
        keys.clear();
        lmap.clear();
        ops.clear();
        auto add = [&](int key) {
          if (keypos[key] < 0) { keypos[key] = (int)keys.size(); keys.push_back(key); }
          return keypos[key];
        };
        add(n + i);   // the row's own input: list position 0 after the IN-first reorder below
        deps(i, [&](int j, int slot) {
          if (in_tail(j) && grp[j] == G) {   // substitute j's expression
            const int pj = pos_of[j];
            ops.push_back(Op{pj, slot, (int)lmap.size()});
            for (int e = h.eoff[pj]; e < h.eoff[pj + 1]; ++e)
              lmap.push_back(add(e < h.xoff[pj] ? n + h.eidx[e] : h.eidx[e]));
          } else {
            ops.push_back(Op{add(j), slot, -1});
          }
        });
        // final layout: IN entries first, then X entries (insertion order within each)
        int nin = 0;
        for (int k : keys) nin += k >= n;
        perm.resize(keys.size());
        int a = 0, b = nin;
        for (size_t q = 0; q < keys.size(); ++q) perm[q] = keys[q] >= n ? a++ : b++;
        const int base = (int)h.eidx.size();
        h.rows.push_back(i);
        h.eidx.resize(base + keys.size());
        for (size_t q = 0; q < keys.size(); ++q) h.eidx[base + perm[q]] = keys[q] >= n ? keys[q] - n : keys[q];
        h.xoff.push_back(base + nin);
        h.eoff.push_back(base + (int)keys.size());
        for (const Op& o : ops) {
          h.op_slot.push_back(o.slot);
          if (o.map < 0) {
            h.op_a.push_back(perm[o.a]);
            h.op_map.push_back(-1);
          } else {
            h.op_a.push_back(o.a);
            h.op_map.push_back((int)h.map.size());
            const int lj = h.eoff[o.a + 1] - h.eoff[o.a];
            for (int q = 0; q < lj; ++q) h.map.push_back(perm[lmap[o.map + q]]);
          }
        }
        h.opoff.push_back((int)h.op_a.size());
        for (int k : keys) keypos[k] = -1;
      }
      const long lent = (long)(h.eidx.size() - c_eidx);
      if (l > l0 && (gent + lent > budget || l - l0 >= gmax) && attempt == 0) {
        // over budget: undo this level and start a new merged level with it
        h.rows.resize(c_rows);
        h.eoff.resize(c_rows + 1);
        h.xoff.resize(c_rows);
        h.eidx.resize(c_eidx);
        h.opoff.resize(c_rows + 1);
        h.op_a.resize(c_ops);
        h.op_slot.resize(c_ops);
        h.op_map.resize(c_ops);
        h.map.resize(c_map);
        h.lptr.push_back((int)h.rows.size());
        ++G;
        l0 = l;
        gent = 0;
        continue;
      }
      gent += lent;
      for (int r : levels[l]) by_off[l - l0].push_back(pos_of[r]);
      break;
    }
  }
  h.lptr.push_back((int)h.rows.size());
  if (L == 0) h.lptr.assign(1, 0);
  h.offptr.assign(1, 0);
  for (const auto& v : by_off) {
    h.offpos.insert(h.offpos.end(), v.begin(), v.end());
    h.offptr.push_back((int)h.offpos.size());
  }
}

// Rows of one merged level are independent (in-group dependencies are substituted), so their
// launch order is free: sort each merged level's positions by storage row (the Morton curve), so
// the contiguous position range each XCD gets (xcd_block) is one compact region of the domain and
// the rows sharing gathered source rows run under one L2. Level order within a merged level (the
// build order) spreads every XCD's range over the whole domain.
void sort_merged_by_row(MergeHost& h) {
  const int P = (int)h.rows.size();
  std::vector<int> old_of(P), newpos(P);
  for (size_t G = 0; G + 1 < h.lptr.size(); ++G) {
    const int a = h.lptr[G], b = h.lptr[G + 1];
    for (int p = a; p < b; ++p) old_of[p] = p;
    std::stable_sort(old_of.begin() + a, old_of.begin() + b, [&](int x, int y) { return h.rows[x] < h.rows[y]; });
  }
  for (int q = 0; q < P; ++q) newpos[old_of[q]] = q;
  MergeHost s;
  s.lptr = h.lptr;
  s.map = h.map;   // op_map values index this array; unchanged
  s.rows.resize(P);
  s.xoff.resize(P);
  s.eoff.assign(1, 0);
  s.opoff.assign(1, 0);
  for (int q = 0; q < P; ++q) {
    const int p = old_of[q];
    s.rows[q] = h.rows[p];
    const int base = (int)s.eidx.size();
    s.eidx.insert(s.eidx.end(), h.eidx.begin() + h.eoff[p], h.eidx.begin() + h.eoff[p + 1]);
    s.xoff[q] = base + (h.xoff[p] - h.eoff[p]);
    s.eoff.push_back((int)s.eidx.size());
    for (int o = h.opoff[p]; o < h.opoff[p + 1]; ++o) {
      s.op_slot.push_back(h.op_slot[o]);
      s.op_map.push_back(h.op_map[o]);
      s.op_a.push_back(h.op_map[o] < 0 ? h.op_a[o] : newpos[h.op_a[o]]);   // substitution: a position
    }
    s.opoff.push_back((int)s.op_a.size());
  }
  s.offptr = h.offptr;
  s.offpos.resize(h.offpos.size());
  for (size_t k = 0; k < h.offpos.size(); ++k) s.offpos[k] = newpos[h.offpos[k]];
  h = std::move(s);
}
}  // namespace

void VaduPrecond::Build(const int* nbr, const std::vector<int>& vo, const std::vector<int>& lab,
                        const std::vector<int>& tptr, const std::vector<int>& trow, const std::vector<int>& tslot,
                        int K0, int K) {
  const int n = n_, m = m_;
  K = std::max(0, std::min(K, n));
  K0 = std::max(0, std::min(K0, K));
  K = std::min(K, K0 + kHeadMaxRows);
  K0_ = K0;
  K_ = K;
  DropGraphs();
  use_graph_ = std::getenv("GPBOOST_AMD_NO_GRAPH") == nullptr;   // diagnostics: eager launches (profilers)
  if (const char* e = std::getenv("GPBOOST_AMD_SEG_FORM")) {
    const std::string f(e);
    if (f != "wave" && f != "block") Fatal("GPBOOST_AMD_SEG_FORM must be wave or block (got '%s')", e);
    seg_wave_ = f == "wave";
  }
  auto kk = [&](int p) { return std::min(vo[p], m); };             // entries of storage row p
  auto part = [&](int p) { return vo[p] < K0 ? 0 : (vo[p] < K ? 1 : 2); };
  std::vector<int> ints;    // every index array of the plan, one upload
  std::vector<int> vslot;   // value slots into Bv (-1: zero padding), one gather per factor
  auto put = [&](const std::vector<int>& v) {
    const size_t at = ints.size();
    ints.insert(ints.end(), v.begin(), v.end());
    return at;
  };

  // ---- tail level plan. Lower solve: levels over tail dependencies only (head values are final
  // by then); B^T solve: a tail row's dependents are later Vecchia rows, all in the tail.
  const int nt = n - K;
  std::vector<int> lt(n, 0), lb(n, 0);
  int Lt = 0, Lb = 0;
  for (int ii = K; ii < n; ++ii) {
    const int i = lab[ii];
    int l = 0;
    for (int r = 0; r < kk(i); ++r) {
      const int j = nbr[(size_t)i * m + r];
      if (part(j) == 2) l = std::max(l, lt[j] + 1);
    }
    lt[i] = l;
    Lt = std::max(Lt, l + 1);
  }
  for (int ii = n - 1; ii >= K; --ii) {
    const int i = lab[ii];
    for (int r = 0; r < kk(i); ++r) {
      const int j = nbr[(size_t)i * m + r];
      if (part(j) == 2) lb[j] = std::max(lb[j], lb[i] + 1);
    }
    Lb = std::max(Lb, lb[i] + 1);
  }
  std::vector<std::vector<int>> groups_b(nt > 0 ? Lb : 0), groups_f(nt > 0 ? Lt : 0);
  for (int p = 0; p < n; ++p)
    if (part(p) == 2) {
      groups_b[lb[p]].push_back(p);
      groups_f[lt[p]].push_back(p);
    }
  // merged tail levels: at most g levels per launch (GPBOOST_AMD_TAIL_MERGE, 1 = the plain level
  // schedule) and at most `budget` entries per launch (GPBOOST_AMD_TAIL_BUDGET)
  // (n = 100k, m = 30, t = 51, per application: g = 1 1.10 ms, g = 2 0.83, g = 3 0.79, g = 4 0.82,
  // g = 8 1.05; g <= 16 with 150k entries 0.78 — beyond ~3 levels the fill's gather bytes, not the
  // launches, set the time)
  int g = 16;
  if (const char* e = std::getenv("GPBOOST_AMD_TAIL_MERGE")) {
    g = std::atoi(e);
    if (g < 1 || g > 64) Fatal("GPBOOST_AMD_TAIL_MERGE must be 1..64 (got '%s')", e);
  }
  long budget = 150000;
  if (const char* e = std::getenv("GPBOOST_AMD_TAIL_BUDGET")) {
    budget = std::atol(e);
    if (budget < 1) Fatal("GPBOOST_AMD_TAIL_BUDGET must be >= 1 (got '%s')", e);
  }
  merge_g_ = g;
  {
    MergeHost mb, ml;
    auto tail = [&](int j) { return part(j) == 2; };
    build_merged(
        n, budget, g, groups_b, [&](int j, auto f) { for (int e = tptr[j]; e < tptr[j + 1]; ++e) f(trow[e], tslot[e]); }, tail,
        mb);
    build_merged(
        n, budget, g, groups_f, [&](int i, auto f) { for (int r = 0; r < kk(i); ++r) f(nbr[(size_t)i * m + r], i * m + r); },
        tail, ml);
    // launch order inside a merged level (GPBOOST_AMD_TAIL_ORDER=level keeps the build's level order)
    const char* tord = std::getenv("GPBOOST_AMD_TAIL_ORDER");
    if (tord && std::string(tord) != "level" && std::string(tord) != "row")
      Fatal("GPBOOST_AMD_TAIL_ORDER must be row or level (got '%s')", tord);
    if (!tord || std::string(tord) == "row") {
      sort_merged_by_row(mb);
      sort_merged_by_row(ml);
    }
    std::vector<int> mint;
    MergeHost* hs[2] = {&mb, &ml};
    size_t o[2][10];
    size_t nval = 0, v0[2];
    for (int w = 0; w < 2; ++w) {
      const MergeHost& h = *hs[w];
      const std::vector<int>* arrs[10] = {&h.rows, &h.eoff, &h.xoff, &h.eidx, &h.opoff, &h.op_a, &h.op_slot,
                                          &h.op_map, &h.map, &h.offpos};
      for (int a = 0; a < 10; ++a) {
        o[w][a] = mint.size();
        mint.insert(mint.end(), arrs[a]->begin(), arrs[a]->end());
      }
      v0[w] = nval;
      nval += h.eidx.size();
    }
    d_mint_.alloc(std::max<size_t>(mint.size(), 1));
    d_mval_.alloc(std::max<size_t>(nval, 1));
    if (!mint.empty())
      HIP_CHECK(hipMemcpyAsync(d_mint_.get(), mint.data(), sizeof(int) * mint.size(), hipMemcpyHostToDevice, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    for (int w = 0; w < 2; ++w) {
      MergedSolve& ms = w == 0 ? mt_bt_ : mt_low_;
      const MergeHost& h = *hs[w];
      const int* I = d_mint_.get();
      ms.npos = (int)h.rows.size();
      ms.lptr = h.lptr;
      ms.offptr = h.offptr;
      ms.rows = I + o[w][0];
      ms.eoff = I + o[w][1];
      ms.xoff = I + o[w][2];
      ms.eidx = I + o[w][3];
      ms.opoff = I + o[w][4];
      ms.op_a = I + o[w][5];
      ms.op_slot = I + o[w][6];
      ms.op_map = I + o[w][7];
      ms.map = I + o[w][8];
      ms.offpos = I + o[w][9];
      ms.eval = d_mval_.get() + v0[w];
    }
    tail_entries_ = (long)nval;
    d_mcoef_.alloc(std::max<size_t>(hs[1]->eidx.size(), 1));

    // persistent tail form: device level boundaries and entry rows tagged with kTailBit where an
    // X entry's row is a tail row (read from the padded copy), per solve
    tail_persist_ = false;
    if (const char* e = std::getenv("GPBOOST_AMD_TAIL_FORM")) {
      const std::string f(e);
      if (f != "persist" && f != "launch") Fatal("GPBOOST_AMD_TAIL_FORM must be persist or launch (got '%s')", e);
      tail_persist_ = f == "persist";
    }
    if (tail_persist_) {
      int W = std::min(64, tail_persist_max_w());
      if (const char* e = std::getenv("GPBOOST_AMD_TAIL_W")) W = std::atoi(e);
      if (W < 1 || W > tail_persist_max_w())
        Fatal("GPBOOST_AMD_TAIL_W: %d workgroups per XCD group, at most %d resident", W, tail_persist_max_w());
      std::vector<int> pint;
      size_t po[2][2];
      for (int w = 0; w < 2; ++w) {
        const MergeHost& h = *hs[w];
        po[w][0] = pint.size();
        pint.insert(pint.end(), h.lptr.begin(), h.lptr.end());
        po[w][1] = pint.size();
        for (size_t p = 0; p < h.rows.size(); ++p)
          for (int q = h.eoff[p]; q < h.eoff[p + 1]; ++q) {
            const int r = h.eidx[q];
            pint.push_back(q >= h.xoff[p] && part(r) == 2 ? (r | kTailBit) : r);
          }
      }
      d_pint_.alloc(std::max<size_t>(pint.size(), 1));
      HIP_CHECK(hipMemcpy(d_pint_.get(), pint.data(), sizeof(int) * pint.size(), hipMemcpyHostToDevice));
      for (int w = 0; w < 2; ++w) {
        TailPersist& tp = w == 0 ? tp_bt_ : tp_low_;
        tp.lptr = d_pint_.get() + po[w][0];
        tp.nL = (int)hs[w]->lptr.size() - 1;
        tp.eidx_p = d_pint_.get() + po[w][1];
        tp.W = W;
      }
      for (int sl = 0; sl < kSlots; ++sl) {
        Tp_[sl].release();
        ctr_[sl].alloc((size_t)9 * std::max(1, tp_bt_.nL + tp_low_.nL));
      }
    }
  }

  // ---- head 1 segment [K0, K): slots = Vecchia index - K0, dependencies inside the segment
  const int KS = K - K0;
  struct SegArrays {
    std::vector<int> rec, eidx, slot, ooff{0}, oidx, oslot, pend;
    std::vector<int> wmeta, wrec, widx, wslot;   // one-wave form (SegWave): meta as 4 ints per pass
  };
  auto build_seg = [&](bool lower) {
    SegArrays h;
    std::vector<int> lev(KS, 0);
    std::vector<std::vector<int>> deps(KS), dslot(KS);
    for (int v = 0; v < KS; ++v) {
      const int p = lab[K0 + v];
      if (lower) {
        for (int r = 0; r < kk(p); ++r) {
          const int j = nbr[(size_t)p * m + r];
          if (part(j) == 1) { deps[v].push_back(vo[j] - K0); dslot[v].push_back(p * m + r); }
        }
      } else {
        for (int e = tptr[p]; e < tptr[p + 1]; ++e)
          if (part(trow[e]) == 1) { deps[v].push_back(vo[trow[e]] - K0); dslot[v].push_back(tslot[e]); }
      }
    }
    int L = 0;
    for (int s = 0; s < KS; ++s) {   // lower: ascending Vecchia index; B^T: descending
      const int v = lower ? s : KS - 1 - s;
      int l = 0;
      for (int d : deps[v]) l = std::max(l, lev[d] + 1);
      lev[v] = l;
      L = std::max(L, l + 1);
    }
    std::vector<std::vector<int>> byl(L);
    for (int s = 0; s < KS; ++s) {
      const int v = lower ? s : KS - 1 - s;
      byl[lev[v]].push_back(v);
    }
    // one-wave form: per level, rows by lane-group class lg (2^lg lanes, each <= kSegSteps entries
    // of the row's own input + dependencies), longest first, up to 64 >> lg rows per pass; steps
    // padded to a multiple of 8 (padding: slot KS, coefficient 0)
    for (const auto& rows : byl) {
      std::vector<std::vector<int>> cls(7);
      for (int v : rows) {
        const int c = 1 + (int)deps[v].size();
        int lg = 0;
        while ((kSegSteps << lg) < c) ++lg;
        if (lg > 6) Fatal("VADU segment row with %d entries exceeds the one-wave plan (%d)", c, kSegSteps << 6);
        cls[lg].push_back(v);
      }
      for (int lg = 0; lg <= 6; ++lg) {
        auto& cv = cls[lg];
        std::stable_sort(cv.begin(), cv.end(), [&](int x, int y) { return deps[x].size() > deps[y].size(); });
        const int G = 1 << lg, per = 64 >> lg;
        for (size_t r0 = 0; r0 < cv.size(); r0 += per) {
          const int nr = (int)std::min<size_t>(per, cv.size() - r0);
          int L = 0;
          for (int r = 0; r < nr; ++r) L = std::max(L, (int)(1 + deps[cv[r0 + r]].size() + G - 1) / G);
          L = (L + 7) / 8 * 8;
          const int off = (int)(h.widx.size() / 64);
          const int q = (int)(h.wmeta.size() / 4);
          h.wmeta.insert(h.wmeta.end(), {off, L, lg, 0});
          h.wrec.resize((size_t)(q + 1) * 64, -1);
          h.widx.resize((size_t)(off + L) * 64, KS * 8);
          h.wslot.resize((size_t)(off + L) * 64, -1);
          for (int r = 0; r < nr; ++r) {
            const int v = cv[r0 + r];
            h.wrec[(size_t)q * 64 + r * G] = v;
            const int c = 1 + (int)deps[v].size();
            for (int e = 0; e < c; ++e) {   // e = 0: the row's own input, coefficient -1
              const int k = e / G, lane = r * G + e % G;
              const size_t at = (size_t)(off + k) * 64 + lane;
              h.widx[at] = (e == 0 ? v : deps[v][e - 1]) * 8;
              h.wslot[at] = e == 0 ? -2 : dslot[v][e - 1];
            }
          }
        }
      }
    }
    const int E = kHeadEpl;
    auto nslots = [&](int v) {   // 1, 2 or 4 slots of kHeadG lanes (rows beyond 4 slots overflow)
      const int c = (int)deps[v].size();
      return c <= kHeadG * E ? 1 : c <= 2 * kHeadG * E ? 2 : 4;
    };
    for (auto rows : byl) {
      // widest rows first: power-of-two sizes in descending order stay aligned in a pass
      std::stable_sort(rows.begin(), rows.end(), [&](int x, int y) { return nslots(x) > nslots(y); });
      size_t q = 0;
      while (q < rows.size()) {   // one pass
        const size_t r_pass = h.rec.size();
        h.rec.resize(r_pass + kHeadRowsPerPass, KS);
        h.ooff.resize(r_pass + kHeadRowsPerPass + 1, (int)h.oidx.size());
        h.eidx.resize((r_pass + kHeadRowsPerPass) * E * kHeadG, 0);
        h.slot.resize((r_pass + kHeadRowsPerPass) * E * kHeadG, -1);
        int used = 0;
        while (q < rows.size() && used + nslots(rows[q]) <= kHeadRowsPerPass) {
          const int v = rows[q], ns = nslots(v), GL = ns * kHeadG;
          const int lg = ns == 1 ? 0 : ns == 2 ? 1 : 2;
          const size_t r0 = r_pass + used;
          const int cnt = (int)deps[v].size();
          const bool over = cnt > GL * E;
          for (int sub = 0; sub < ns; ++sub)
            h.rec[r0 + sub] = (int)((over ? 0x80000000u : 0u) | ((unsigned)sub << 18) | ((unsigned)lg << 16) |
                                    (unsigned)(sub == 0 ? v : KS));
          for (int e = 0; e < std::min(cnt, GL * E); ++e) {   // entry e -> group lane e % GL, k = e / GL
            const int gl = e % GL, k = e / GL;
            const size_t at = ((r0 + gl / kHeadG) * E + k) * kHeadG + gl % kHeadG;
            h.eidx[at] = deps[v][e];
            h.slot[at] = dslot[v][e];
          }
          h.ooff[r0] = (int)h.oidx.size();
          for (int e = GL * E; e < cnt; ++e) { h.oidx.push_back(deps[v][e]); h.oslot.push_back(dslot[v][e]); }
          for (int sub = 1; sub <= ns; ++sub) h.ooff[r0 + sub] = (int)h.oidx.size();
          used += ns;
          ++q;
        }
        for (size_t r = r_pass + used; r <= r_pass + kHeadRowsPerPass; ++r) h.ooff[r] = (int)h.oidx.size();
        h.pend.push_back(q >= rows.size() ? 1 : 0);   // last pass of its level: barrier after it
      }
    }
    return h;
  };
  SegArrays sl = build_seg(true), sb = build_seg(false);
  std::vector<int> hrow(KS);
  for (int v = 0; v < KS; ++v) hrow[v] = lab[K0 + v];
  const size_t o_hrow = put(hrow);
  size_t o_s[2][8], v_s[2][3];
  for (int w = 0; w < 2; ++w) {
    SegArrays& h = w == 0 ? sl : sb;
    o_s[w][0] = put(h.rec);
    o_s[w][1] = put(h.eidx);
    o_s[w][2] = put(h.oidx);
    o_s[w][3] = put(h.ooff);
    o_s[w][4] = put(h.pend);
    while (ints.size() % 4) ints.push_back(0);   // int4 alignment of the pass metas
    o_s[w][5] = put(h.wmeta);
    o_s[w][6] = put(h.wrec);
    o_s[w][7] = put(h.widx);
    v_s[w][0] = vslot.size();
    vslot.insert(vslot.end(), h.slot.begin(), h.slot.end());
    v_s[w][1] = vslot.size();
    vslot.insert(vslot.end(), h.oslot.begin(), h.oslot.end());
    v_s[w][2] = vslot.size();
    vslot.insert(vslot.end(), h.wslot.begin(), h.wslot.end());
  }

  // ---- partial sums across parts
  struct PartArrays { std::vector<int> row, off{0}, idx, slot; };
  PartArrays th, p10, p01;
  for (int v = 0; v < K; ++v) {   // B^T: tail dependents of every head row
    const int j = lab[v];
    th.row.push_back(j);
    for (int e = tptr[j]; e < tptr[j + 1]; ++e)
      if (part(trow[e]) == 2) { th.idx.push_back(trow[e]); th.slot.push_back(tslot[e]); }
    th.off.push_back((int)th.idx.size());
  }
  if (KS > 0) {
    for (int v = 0; v < K0; ++v) {   // B^T: head-1 dependents of every head-0 row
      const int j = lab[v];
      p10.row.push_back(j);
      for (int e = tptr[j]; e < tptr[j + 1]; ++e)
        if (part(trow[e]) == 1) { p10.idx.push_back(trow[e]); p10.slot.push_back(tslot[e]); }
      p10.off.push_back((int)p10.idx.size());
    }
    if (K0 > 0) {
      for (int v = 0; v < KS; ++v) {   // lower: head-0 neighbours of every head-1 row
        const int p = lab[K0 + v];
        p01.row.push_back(p);
        for (int r = 0; r < kk(p); ++r) {
          const int j = nbr[(size_t)p * m + r];
          if (part(j) == 0) { p01.idx.push_back(j); p01.slot.push_back(p * m + r); }
        }
        p01.off.push_back((int)p01.idx.size());
      }
    }
  }
  size_t o_p[3][3], v_p[3];
  PartArrays* pa[3] = {&th, &p10, &p01};
  for (int w = 0; w < 3; ++w) {
    o_p[w][0] = put(pa[w]->row);
    o_p[w][1] = put(pa[w]->off);
    o_p[w][2] = put(pa[w]->idx);
    v_p[w] = vslot.size();
    vslot.insert(vslot.end(), pa[w]->slot.begin(), pa[w]->slot.end());
  }

  // ---- dense head: storage rows of head-0 slots, and per entry (i, r) of its rows the Vecchia
  // column of B_00 (-1: padding) next to the value slot
  std::vector<int> h0row(K0), dcol((size_t)K0 * m, -1), dslot0((size_t)K0 * m, -1);
  for (int v = 0; v < K0; ++v) {
    const int p = lab[v];
    h0row[v] = p;
    for (int r = 0; r < kk(p); ++r) {
      dcol[(size_t)v * m + r] = vo[nbr[(size_t)p * m + r]];
      dslot0[(size_t)v * m + r] = p * m + r;
    }
  }
  const size_t o_h0row = put(h0row), o_dcol = put(dcol);
  const size_t v_d0 = vslot.size();
  vslot.insert(vslot.end(), dslot0.begin(), dslot0.end());

  // ---- upload, then point the plan structs into the two arrays
  d_int_.alloc(std::max<size_t>(ints.size(), 1));
  d_slot_.alloc(std::max<size_t>(vslot.size(), 1));
  d_val_.alloc(std::max<size_t>(vslot.size(), 1));
  if (!ints.empty())
    HIP_CHECK(hipMemcpyAsync(d_int_.get(), ints.data(), sizeof(int) * ints.size(), hipMemcpyHostToDevice, s_));
  if (!vslot.empty())
    HIP_CHECK(hipMemcpyAsync(d_slot_.get(), vslot.data(), sizeof(int) * vslot.size(), hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  nslot_ = (int)vslot.size();
  const int* I = d_int_.get();
  const double* V = d_val_.get();
  for (int w = 0; w < 2; ++w) {
    HeadSolve& h = w == 0 ? seg_low_ : seg_bt_;
    const SegArrays& a = w == 0 ? sl : sb;
    h.K = KS;
    h.npass = (int)(a.rec.size() / kHeadRowsPerPass);
    h.hrow = I + o_hrow;
    h.rec = I + o_s[w][0];
    h.eidx = I + o_s[w][1];
    h.oidx = I + o_s[w][2];
    h.ooff = I + o_s[w][3];
    h.pend = I + o_s[w][4];
    h.eval = V + v_s[w][0];
    h.oval = V + v_s[w][1];
    SegWave& sw = w == 0 ? segw_low_ : segw_bt_;
    sw.K = KS;
    sw.npass = (int)(a.wmeta.size() / 4);
    sw.hrow = I + o_hrow;
    sw.meta = reinterpret_cast<const int4*>(I + o_s[w][5]);
    sw.rec = I + o_s[w][6];
    sw.eidx = I + o_s[w][7];
    sw.eval = V + v_s[w][2];
  }
  PartialList* pl[3] = {&p_th_, &p_10_, &p_01_};
  for (int w = 0; w < 3; ++w) {
    pl[w]->rows = (int)pa[w]->row.size();
    pl[w]->row = I + o_p[w][0];
    pl[w]->eoff = I + o_p[w][1];
    pl[w]->eidx = I + o_p[w][2];
    pl[w]->eval = V + v_p[w];
  }
  dh_.K0 = K0;
  dh_.m = m;
  dh_.row = I + o_h0row;
  dh_.col = I + o_dcol;
  dh_.val = V + v_d0;
  if (KS > 0) set_vadu_head_lds_limit(KS);
  // ---- dense head buffers (G's strict upper triangle stays zero: TRTRI writes lower blocks only)
  ld0_ = ((K0 + 63) / 64) * 64;
  dh_.ld = ld0_;
  if (K0 > 0) {
    const size_t nn = (size_t)ld0_ * ld0_;
    Bd_.alloc(nn);
    G_.alloc(nn);
    GT_.alloc(nn);
    T_.alloc((size_t)ld0_ * (ld0_ / 2 + 64));
    HIP_CHECK(hipMemsetAsync(G_.get(), 0, nn * sizeof(double), s_));
    HIP_CHECK(hipStreamSynchronize(s_));
  }
}

void VaduPrecond::Refresh(const double* Bv) {
  launch_gather(nslot_, d_slot_.get(), Bv, d_val_.get(), s_);
  launch_merged_numeric(mt_bt_, Bv, s_);
  launch_merged_numeric(mt_low_, Bv, s_);
  if (dw_) launch_merged_scale(mt_low_, dw_, d_mcoef_.get(), s_);
  if (K0_ > 0) dense_head_factor(dh_, Bd_.get(), G_.get(), GT_.get(), T_.get(), s_);
}

void VaduPrecond::SetDiag(const double* dw) {
  if (dw != dw_) DropGraphs();   // the captured launches hold the pointer
  dw_ = dw;
  launch_merged_scale(mt_low_, dw_, d_mcoef_.get(), s_);   // dw's values change with every Newton step
}

void VaduPrecond::DenseApply(const double* X0, double* Z, int t, hipStream_t st, double* S) {
  // S holds >= 2 ld0_ t doubles (the compact head-0 block, then the scaled G^T product)
  launch_dense_head_apply(dh_, G_.get(), GT_.get(), dw_, X0, S, Z, t, st);
}

void VaduPrecond::SegSolve(bool lower, const double* in, const double* dw, double* X, int t, hipStream_t st) {
  if (seg_wave_) launch_vadu_seg_wave(lower ? segw_low_ : segw_bt_, in, dw, X, t, st);
  else launch_vadu_head(lower ? seg_low_ : seg_bt_, in, dw, X, t, st);
}

void VaduPrecond::TailSolve(bool lower, const double* R, double* Xt, double* Z, int t, hipStream_t st, int slot) {
  const MergedSolve& ms = lower ? mt_low_ : mt_bt_;
  if (TailPersistOn(t)) {
    // B^T solve: IN = R, values to Xt; lower solve: IN = Xt, head rows of Z final, values to Z
    unsigned* ctr = ctr_[slot].get() + (lower ? (size_t)9 * tp_bt_.nL : 0);
    if (lower) launch_tail_persist(ms, tp_low_, ctr, d_mcoef_.get(), Xt, Z, Tp_[slot].get(), Z, t, st);
    else launch_tail_persist(ms, tp_bt_, ctr, ms.eval, R, Xt, Tp_[slot].get(), Xt, t, st);
    return;
  }
  for (int L = 0; L + 1 < (int)ms.lptr.size(); ++L)
    launch_merged_level(ms, L, lower ? d_mcoef_.get() : ms.eval, lower ? Xt : R, lower ? Z : Xt, t, st);
}

void VaduPrecond::Record(const double* R, double* Z, double* Xt, int t, hipStream_t st, double* S, int slot) {
  const bool seg = K_ > K0_;
  TailSolve(false, R, Xt, Z, t, st, slot);
  // the last partial sum over the head-0 rows also stores them compactly for the dense products
  double* x0 = K0_ > 0 ? S : nullptr;
  if (K_ > 0) launch_vadu_partial(p_th_, R, nullptr, Xt, Xt, t, st, seg ? nullptr : x0, K0_);
  if (seg) SegSolve(false, Xt, nullptr, Xt, t, st);
  if (K0_ > 0) {
    if (seg) launch_vadu_partial(p_10_, nullptr, nullptr, Xt, Xt, t, st, x0, K0_);
    DenseApply(x0, Z, t, st, S);
  }
  if (seg) {
    if (K0_ > 0) {
      launch_vadu_partial(p_01_, Xt, dw_, Z, Z, t, st);
      SegSolve(true, Z, nullptr, Z, t, st);
    } else {
      SegSolve(true, Xt, dw_, Z, t, st);
    }
  }
  TailSolve(true, R, Xt, Z, t, st, slot);
}

double* VaduPrecond::Scratch(int slot, int t) {
  if (slot < 0 || slot >= kSlots) Fatal("VADU preconditioner scratch slot %d out of range", slot);
  if (K0_ > 0 && S_[slot].size() < (size_t)2 * ld0_ * t) {   // sized before any capture that uses it
    HIP_CHECK(hipDeviceSynchronize());   // eager launches in flight may still use the old scratch
    DropGraphs();
    S_[slot].alloc((size_t)2 * ld0_ * t);
  }
  if (TailPersistOn(t) && Tp_[slot].size() == 0) {
    HIP_CHECK(hipDeviceSynchronize());
    DropGraphs();
    Tp_[slot].alloc((size_t)n_ * kTailPad);
  }
  return S_[slot].get();
}

void VaduPrecond::Apply(const double* R, double* Z, double* Xt, int t, hipStream_t st, int slot) {
  if (!dw_) Fatal("VADU preconditioner applied before SetDiag");
  if (!st) st = s_;
  double* S = Scratch(slot, t);
  if (!use_graph_) {
    Record(R, Z, Xt, t, st, S, slot);
    return;
  }
  for (const GraphEntry& g : graphs_) {
    if (g.key[0] == R && g.key[1] == Z && g.key[2] == Xt && g.t == t && g.slot == slot) {
      HIP_CHECK(hipGraphLaunch(g.exec, st));
      return;
    }
  }
  hipGraph_t graph;
  HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  Record(R, Z, Xt, t, st, S, slot);
  HIP_CHECK(hipStreamEndCapture(st, &graph));
  GraphEntry e{{R, Z, Xt}, t, slot, nullptr};
  HIP_CHECK(hipGraphInstantiate(&e.exec, graph, nullptr, nullptr, 0));
  HIP_CHECK(hipGraphDestroy(graph));
  graphs_.push_back(e);
  HIP_CHECK(hipGraphLaunch(e.exec, st));
}

void VaduPrecond::TimeParts(const double* R, double* Z, double* Xt, int t, int reps) {
  double* S = Scratch(0, t);
  hipEvent_t a, b;
  HIP_CHECK(hipEventCreate(&a));
  HIP_CHECK(hipEventCreate(&b));
  const bool seg = K_ > K0_;
  auto part = [&](const char* name, auto fn) {
    float ms = 0.f;
    HIP_CHECK(hipEventRecord(a, s_));
    for (int r = 0; r < reps; ++r) fn();
    HIP_CHECK(hipEventRecord(b, s_));
    HIP_CHECK(hipEventSynchronize(b));
    HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    std::fprintf(stderr, "[precond parts t=%d] %-11s %.4f ms\n", t, name, ms / reps);
  };
  part("tail_bt", [&] { TailSolve(false, R, Xt, Z, t, s_, 0); });
  part("part_th", [&] { launch_vadu_partial(p_th_, R, nullptr, Xt, Xt, t, s_, seg ? nullptr : S, K0_); });
  if (seg) part("seg_bt", [&] { SegSolve(false, Xt, nullptr, Xt, t, s_); });
  if (K0_ > 0 && seg) part("part_10", [&] { launch_vadu_partial(p_10_, nullptr, nullptr, Xt, Xt, t, s_, S, K0_); });
  if (K0_ > 0) part("dense", [&] { DenseApply(S, Z, t, s_, S); });
  if (K0_ > 0 && seg) part("part_01", [&] { launch_vadu_partial(p_01_, Xt, dw_, Z, Z, t, s_); });
  if (seg) part("seg_low", [&] { SegSolve(true, Z, nullptr, Z, t, s_); });
  part("tail_low", [&] { TailSolve(true, R, Xt, Z, t, s_, 0); });
  if (TailPersistOn(t)) {   // the persistent form without its barriers / without its gathers (timing only)
    for (int d = 1; d <= 2; ++d) {
      tp_bt_.diag = d;
      part(d == 1 ? "tail_bt_nobar" : "tail_bt_nogath", [&] { TailSolve(false, R, Xt, Z, t, s_, 0); });
    }
    tp_bt_.diag = 0;
  }
  std::fprintf(stderr,
               "[precond parts t=%d] K0=%d K=%d passes bt=%d low=%d tail merged levels bt=%d low=%d (g=%d, %ld entries) "
               "launches=%d\n",
               t, K0_, K_, seg_wave_ ? segw_bt_.npass : seg_bt_.npass, seg_wave_ ? segw_low_.npass : seg_low_.npass, tail_levels_bt(), tail_levels_lower(), merge_g_, tail_entries_,
               launches());
  HIP_CHECK(hipEventDestroy(a));
  HIP_CHECK(hipEventDestroy(b));
}

}  // namespace gpb_amd
