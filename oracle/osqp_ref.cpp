// osqp_ref.cpp -- CPU ORACLE / BASELINE (test infrastructure, never shipped, never on the
// product path).  Float64 restatement of what the reference executes per MPC tick:
//
//   CentroidalMPC.solve_QP (convex_mpc/centroidal_mpc.py:69-120) builds the QP data
//   (_update_sparse_matrix :235-285, _compute_bounds :122-176, friction :324-359,
//   H :178-201) and calls CasADi 3.6.7's conic plugin "osqp" (:213, :98) with OPTS (:20-36):
//   eps_abs = eps_rel = 1e-4, max_iter 1000, polish off, adaptive_rho on with interval 25,
//   check_termination 10, scaling 5, scaled_termination on, warm start primal + dual.
//
// CasADi and OSQP are not installed here; this file restates the published
// OSQP 0.6 algorithm (operator splitting with Ruiz equilibration + cost scaling, rho vector
// with RHO_MIN on free rows and 1e3 rho on equality rows, alpha relaxation, adaptive rho,
// scaled termination) on CasADi's data layout for conic/osqp: constraints [I; A] with
// [lbx; lba] <= [I; A] w <= [ubx; uba].  The quasi-definite KKT
// [P + sigma I, A'; A, -diag(1/rho)] is factored by a sparse LDL' (up-looking, elimination
// tree; the algorithm of QDLDL, OSQP's default linear system solver) under a minimum-degree
// ordering (OSQP uses AMD; the ordering only changes fill, not the solution).
// Primal/dual infeasibility detection is omitted: the reference QP is always feasible
// (states free, fx = fy = 0, fz = fz_min satisfies every stance row).
//
// Build: see oracle/Makefile (g++ -O2 -fopenmp -shared).
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <set>
#include <vector>

namespace {

constexpr double kInf = 1e30;          // OSQP_INFTY
constexpr double kMinScaling = 1e-4;   // MIN_SCALING
constexpr double kMaxScaling = 1e4;    // MAX_SCALING
constexpr double kRhoMin = 1e-6;       // RHO_MIN
constexpr double kRhoMax = 1e6;        // RHO_MAX
constexpr double kRhoTol = 1e-4;       // RHO_TOL (equality detection)
constexpr double kRhoEqOverIneq = 1e3; // RHO_EQ_OVER_RHO_INEQ
constexpr double kDivTol = 1e-30;      // DIVISION_TOL

struct Csc {  // compressed sparse column
  int m = 0, n = 0;
  std::vector<int> p, i;
  std::vector<double> x;
};

// ---------------------------------------------------------------------------------------
// QP data in the reference layout (centroidal_mpc.py:122-359), CasADi conic -> OSQP form
// ---------------------------------------------------------------------------------------
struct Problem {
  int N, n, m;  // vars, rows of [I; A]
  Csc P;        // upper triangle of H (diagonal)
  Csc A;        // [I; A_ref]  (m x n)
  std::vector<double> q, l, u;
};

void build_problem(int N, const double* Q, const double* R, double mu, double fz_min,
                   const double* Ad, const double* Bd, const double* gd, const double* x0,
                   const double* xref /* [N][12] */, const uint8_t* ct /* [4][N] */,
                   Problem& pr) {
  const int NX = 12, NU = 12;
  const int nv = N * (NX + NU);
  const int neq = N * NX, nfr = 16 * N;
  const int mA = neq + nfr;
  pr.N = N;
  pr.n = nv;
  pr.m = nv + mA;
  // H = diag(2Q x N, 2R x N)  (centroidal_mpc.py:184-200)
  pr.P.m = pr.P.n = nv;
  pr.P.p.resize(nv + 1);
  pr.P.i.resize(nv);
  pr.P.x.resize(nv);
  for (int j = 0; j < nv; ++j) {
    pr.P.p[j] = j;
    pr.P.i[j] = j;
    pr.P.x[j] = (j < N * NX) ? 2.0 * Q[j % NX] : 2.0 * R[(j - N * NX) % NU];
  }
  pr.P.p[nv] = nv;
  // A_ref by columns: x_j columns (j = 0..N-1 -> x_{j+1}): +I in row block j, -Ad in row
  // block j+1; u_k columns: -Bd_k in row block k, friction rows.  A_total = [I; A_ref].
  std::vector<std::vector<std::pair<int, double>>> cols(nv);
  for (int c = 0; c < nv; ++c) cols[c].push_back({c, 1.0});  // identity (bounds) rows
  const int r0 = nv;
  for (int k = 0; k < N; ++k) {  // column block of x_{k+1}
    for (int jj = 0; jj < NX; ++jj) {
      const int c = k * NX + jj;
      cols[c].push_back({r0 + k * NX + jj, 1.0});
      if (k + 1 < N)
        for (int ii = 0; ii < NX; ++ii)  // structural: SX blocks are dense (5168 nnz)
          cols[c].push_back({r0 + (k + 1) * NX + ii, -Ad[ii * NX + jj]});
    }
  }
  for (int k = 0; k < N; ++k) {  // u_k columns
    for (int jj = 0; jj < NU; ++jj) {
      const int c = N * NX + k * NU + jj;
      for (int ii = 0; ii < NX; ++ii) cols[c].push_back({r0 + k * NX + ii, -Bd[(k * NX + ii) * NU + jj]});
      const int leg = jj / 3, ax = jj % 3;
      const int fr = r0 + neq + (k * 4 + leg) * 4;
      if (ax == 0) { cols[c].push_back({fr + 0, 1.0}); cols[c].push_back({fr + 1, -1.0}); }
      if (ax == 1) { cols[c].push_back({fr + 2, 1.0}); cols[c].push_back({fr + 3, -1.0}); }
      if (ax == 2) for (int f = 0; f < 4; ++f) cols[c].push_back({fr + f, -mu});
    }
  }
  pr.A.m = pr.m;
  pr.A.n = nv;
  pr.A.p.assign(nv + 1, 0);
  pr.A.i.clear();
  pr.A.x.clear();
  for (int c = 0; c < nv; ++c) {
    std::sort(cols[c].begin(), cols[c].end());
    pr.A.p[c + 1] = pr.A.p[c] + (int)cols[c].size();
    for (auto& e : cols[c]) { pr.A.i.push_back(e.first); pr.A.x.push_back(e.second); }
  }
  // g = [vec(-2 Q xref); 0]  (centroidal_mpc.py:248-253); xref[k] is column k
  pr.q.assign(nv, 0.0);
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < NX; ++i) pr.q[k * NX + i] = -2.0 * Q[i] * xref[k * NX + i];
  // bounds: [lbx; lba], [ubx; uba]
  pr.l.assign(pr.m, -kInf);
  pr.u.assign(pr.m, kInf);
  for (int k = 0; k < N; ++k)  // _compute_bounds (centroidal_mpc.py:122-176)
    for (int leg = 0; leg < 4; ++leg) {
      const int base = N * NX + k * NU + 3 * leg;
      if (ct[leg * N + k]) {
        pr.l[base + 2] = std::max(pr.l[base + 2], fz_min);
      } else {
        for (int a = 0; a < 3; ++a) pr.l[base + a] = pr.u[base + a] = 0.0;
      }
    }
  for (int k = 0; k < N; ++k)  // beq (centroidal_mpc.py:257-261)
    for (int i = 0; i < NX; ++i) {
      double v = gd[i];
      if (k == 0) for (int j = 0; j < NX; ++j) v += Ad[i * NX + j] * x0[j];
      pr.l[r0 + k * NX + i] = pr.u[r0 + k * NX + i] = v;
    }
  for (int k = 0; k < N; ++k)  // friction rows (centroidal_mpc.py:264-283)
    for (int leg = 0; leg < 4; ++leg)
      if (ct[leg * N + k])
        for (int f = 0; f < 4; ++f) pr.u[r0 + neq + (k * 4 + leg) * 4 + f] = 0.0;
}

// ---------------------------------------------------------------------------------------
// sparse LDL' (elimination tree, up-looking) on a fixed symmetric pattern
// ---------------------------------------------------------------------------------------
struct Ldl {
  int n = 0;
  std::vector<int> perm, pinv;   // new -> old, old -> new
  Csc K;                         // permuted upper triangle (pattern fixed)
  std::vector<int> kmap_P, kmap_A, kmap_rho;  // positions of P, A, -1/rho entries in K.x
  std::vector<int> etree, Lnz, Lp, Li;
  std::vector<double> Lx, D, Dinv;
  // scratch
  std::vector<int> iwork, flag, yidx, ebuf, next;
  std::vector<double> yv, bw;
};

// minimum-degree ordering of a symmetric pattern (explicit elimination graph)
std::vector<int> min_degree(int n, const std::vector<std::set<int>>& adj0) {
  std::vector<std::set<int>> adj = adj0;
  std::vector<char> done(n, 0);
  std::vector<int> order;
  order.reserve(n);
  for (int s = 0; s < n; ++s) {
    int best = -1;
    size_t bd = (size_t)-1;
    for (int v = 0; v < n; ++v)
      if (!done[v] && adj[v].size() < bd) { bd = adj[v].size(); best = v; }
    done[best] = 1;
    order.push_back(best);
    std::vector<int> nb(adj[best].begin(), adj[best].end());
    for (int a : nb) adj[a].erase(best);
    for (size_t x = 0; x < nb.size(); ++x)
      for (size_t y = x + 1; y < nb.size(); ++y) {
        adj[nb[x]].insert(nb[y]);
        adj[nb[y]].insert(nb[x]);
      }
    adj[best].clear();
  }
  return order;
}

void ldl_symbolic(Ldl& f, const Problem& pr) {
  const int n = pr.n, m = pr.m, nk = n + m;
  f.n = nk;
  // full symmetric pattern of KKT = [P + sigma I, A'; A, -1/rho]
  std::vector<std::set<int>> adj(nk);
  for (int c = 0; c < n; ++c)
    for (int p = pr.A.p[c]; p < pr.A.p[c + 1]; ++p) {
      const int r = n + pr.A.i[p];
      adj[c].insert(r);
      adj[r].insert(c);
    }
  f.perm = min_degree(nk, adj);
  f.pinv.assign(nk, 0);
  for (int k = 0; k < nk; ++k) f.pinv[f.perm[k]] = k;
  // entries (row, col) in original numbering, upper part after permutation
  struct Ent { int r, c, src, idx; };  // src 0: P diag, 1: A, 2: rho diag
  std::vector<Ent> ents;
  for (int c = 0; c < n; ++c) ents.push_back({c, c, 0, c});
  for (int c = 0; c < n; ++c)
    for (int p = pr.A.p[c]; p < pr.A.p[c + 1]; ++p) ents.push_back({n + pr.A.i[p], c, 1, p});
  for (int r = 0; r < m; ++r) ents.push_back({n + r, n + r, 2, r});
  std::vector<std::vector<std::pair<int, int>>> colent(nk);  // per permuted col: (row, ent)
  for (int e = 0; e < (int)ents.size(); ++e) {
    int i = f.pinv[ents[e].r], j = f.pinv[ents[e].c];
    if (i > j) std::swap(i, j);
    colent[j].push_back({i, e});
  }
  f.K.m = f.K.n = nk;
  f.K.p.assign(nk + 1, 0);
  f.kmap_P.assign(n, 0);
  f.kmap_A.assign(pr.A.i.size(), 0);
  f.kmap_rho.assign(m, 0);
  for (int j = 0; j < nk; ++j) {
    std::sort(colent[j].begin(), colent[j].end());
    for (auto& pe : colent[j]) {
      const int pos = (int)f.K.i.size();
      f.K.i.push_back(pe.first);
      const Ent& e = ents[pe.second];
      if (e.src == 0) f.kmap_P[e.idx] = pos;
      else if (e.src == 1) f.kmap_A[e.idx] = pos;
      else f.kmap_rho[e.idx] = pos;
    }
    f.K.p[j + 1] = (int)f.K.i.size();
  }
  f.K.x.assign(f.K.i.size(), 0.0);
  // elimination tree + column counts
  f.etree.assign(nk, -1);
  f.Lnz.assign(nk, 0);
  f.iwork.assign(nk, -1);
  for (int j = 0; j < nk; ++j) {
    f.iwork[j] = j;
    for (int p = f.K.p[j]; p < f.K.p[j + 1]; ++p) {
      int i = f.K.i[p];
      if (i >= j) continue;
      while (f.iwork[i] != j) {
        if (f.etree[i] == -1) f.etree[i] = j;
        f.Lnz[i]++;
        f.iwork[i] = j;
        i = f.etree[i];
      }
    }
  }
  f.Lp.assign(nk + 1, 0);
  for (int i = 0; i < nk; ++i) f.Lp[i + 1] = f.Lp[i] + f.Lnz[i];
  f.Li.assign(f.Lp[nk], 0);
  f.Lx.assign(f.Lp[nk], 0.0);
  f.D.assign(nk, 0.0);
  f.Dinv.assign(nk, 0.0);
  f.flag.assign(nk, 0);
  f.yidx.assign(nk, 0);
  f.ebuf.assign(nk, 0);
  f.next.assign(nk, 0);
  f.yv.assign(nk, 0.0);
  f.bw.assign(nk, 0.0);
}

// numeric factorization of f.K (up-looking LDL', the QDLDL recurrence)
bool ldl_numeric(Ldl& f) {
  const int n = f.n;
  for (int i = 0; i < n; ++i) { f.flag[i] = 0; f.next[i] = f.Lp[i]; f.yv[i] = 0.0; }
  for (int k = 0; k < n; ++k) {
    int nnzY = 0;
    f.D[k] = 0.0;
    for (int p = f.K.p[k]; p < f.K.p[k + 1]; ++p) {
      const int b = f.K.i[p];
      if (b == k) { f.D[k] = f.K.x[p]; continue; }
      f.yv[b] = f.K.x[p];
      if (!f.flag[b]) {
        int ne = 0;
        int nx = b;
        f.flag[nx] = 1;
        f.ebuf[ne++] = nx;
        nx = f.etree[nx];
        while (nx != -1 && nx < k && !f.flag[nx]) {
          f.flag[nx] = 1;
          f.ebuf[ne++] = nx;
          nx = f.etree[nx];
        }
        while (ne) f.yidx[nnzY++] = f.ebuf[--ne];
      }
    }
    for (int t = nnzY - 1; t >= 0; --t) {
      const int c = f.yidx[t];
      const double yc = f.yv[c];
      const int end = f.next[c];
      for (int j = f.Lp[c]; j < end; ++j) f.yv[f.Li[j]] -= f.Lx[j] * yc;
      f.Li[end] = k;
      const double l = yc * f.Dinv[c];
      f.Lx[end] = l;
      f.D[k] -= yc * l;
      f.next[c]++;
      f.yv[c] = 0.0;
      f.flag[c] = 0;
    }
    if (f.D[k] == 0.0) return false;
    f.Dinv[k] = 1.0 / f.D[k];
  }
  return true;
}

void ldl_solve(Ldl& f, double* x /* permuted in/out */) {
  const int n = f.n;
  for (int i = 0; i < n; ++i)
    for (int j = f.Lp[i]; j < f.Lp[i + 1]; ++j) x[f.Li[j]] -= f.Lx[j] * x[i];
  for (int i = 0; i < n; ++i) x[i] *= f.Dinv[i];
  for (int i = n - 1; i >= 0; --i)
    for (int j = f.Lp[i]; j < f.Lp[i + 1]; ++j) x[i] -= f.Lx[j] * x[f.Li[j]];
}

double inf_norm(const std::vector<double>& v) {
  double m = 0.0;
  for (double a : v) m = std::max(m, fabs(a));
  return m;
}

double limit_scaling(double v) {
  if (v < kMinScaling) return 1.0;
  if (v > kMaxScaling) return kMaxScaling;
  return v;
}

}  // namespace

extern "C" {

struct osqp_ref_settings {
  double Q[12], R[12], mu, fz_min;
  double rho, sigma, alpha, eps_abs, eps_rel, adaptive_rho_tolerance;
  int max_iter, check_termination, adaptive_rho_interval, scaling, scaled_termination;
};

void osqp_ref_default(osqp_ref_settings* s) {
  const double Q[12] = {1, 1, 50, 10, 20, 1, 2, 2, 1, 1, 1, 1};  // centroidal_mpc.py:12
  for (int i = 0; i < 12; ++i) { s->Q[i] = Q[i]; s->R[i] = 1e-5; }  // :13
  s->mu = 0.8;        // :15
  s->fz_min = 10.0;   // :127
  s->rho = 0.1;       // OSQP default
  s->sigma = 1e-6;    // OSQP default
  s->alpha = 1.6;     // OSQP default
  s->eps_abs = 1e-4;  // OPTS :25
  s->eps_rel = 1e-4;  // OPTS :26
  s->adaptive_rho_tolerance = 5.0;  // OSQP default
  s->max_iter = 1000;               // OPTS :27
  s->check_termination = 10;        // OPTS :31
  s->adaptive_rho_interval = 25;    // OPTS :32
  s->scaling = 5;                   // OPTS :33
  s->scaled_termination = 1;        // OPTS :34
}

// Solve B independent instances (layouts as include/cmpc.h, float64).  Cold start per
// instance (the first solve_QP call; warm start applies from the second tick of one robot).
// Outputs w (B, 24N), lam_x (B, 24N), lam_a (B, 28N), status (1 solved, -2 max iter),
// iters.  Returns 0.
int osqp_ref_solve_batch(int B, int N, const double* Ad, const double* Bd, const double* gd,
                         const double* x0, const double* xref, const uint8_t* contact,
                         const osqp_ref_settings* st, double* w_out, double* lam_x_out,
                         double* lam_a_out, int* status, int* iters, int nthreads) {
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
  {
    Problem pr;
    Ldl f;
    bool have_symbolic = false;
#pragma omp for schedule(dynamic, 1)
    for (int b = 0; b < B; ++b) {
      build_problem(N, st->Q, st->R, st->mu, st->fz_min, Ad + (size_t)b * 144,
                    Bd + (size_t)b * N * 144, gd + (size_t)b * 12, x0 + (size_t)b * 12,
                    xref + (size_t)b * N * 12, contact + (size_t)b * 4 * N, pr);
      if (!have_symbolic) { ldl_symbolic(f, pr); have_symbolic = true; }
      const int n = pr.n, m = pr.m;
      // ---- Ruiz equilibration + cost scaling (OSQP scale_data) ----
      std::vector<double> D(n, 1.0), E(m, 1.0), Dt(n), Et(m);
      double c = 1.0;
      Csc P = pr.P, A = pr.A;
      std::vector<double> q = pr.q;
      for (int it = 0; it < st->scaling; ++it) {
        for (int j = 0; j < n; ++j) {
          double cn = 0.0;
          for (int p = P.p[j]; p < P.p[j + 1]; ++p) cn = std::max(cn, fabs(P.x[p]));  // diag P
          for (int p = A.p[j]; p < A.p[j + 1]; ++p) cn = std::max(cn, fabs(A.x[p]));
          Dt[j] = 1.0 / sqrt(limit_scaling(cn));
        }
        std::fill(Et.begin(), Et.end(), 0.0);
        for (int j = 0; j < n; ++j)
          for (int p = A.p[j]; p < A.p[j + 1]; ++p) Et[A.i[p]] = std::max(Et[A.i[p]], fabs(A.x[p]));
        for (int i = 0; i < m; ++i) Et[i] = 1.0 / sqrt(limit_scaling(Et[i]));
        for (int j = 0; j < n; ++j) {
          for (int p = P.p[j]; p < P.p[j + 1]; ++p) P.x[p] *= Dt[P.i[p]] * Dt[j];
          for (int p = A.p[j]; p < A.p[j + 1]; ++p) A.x[p] *= Et[A.i[p]] * Dt[j];
          q[j] *= Dt[j];
          D[j] *= Dt[j];
        }
        for (int i = 0; i < m; ++i) E[i] *= Et[i];
        double mean = 0.0;
        for (int j = 0; j < n; ++j) {
          double cn = 0.0;
          for (int p = P.p[j]; p < P.p[j + 1]; ++p) cn = std::max(cn, fabs(P.x[p]));
          mean += cn;
        }
        mean = limit_scaling(mean / n);
        const double qn = limit_scaling(inf_norm(q));
        const double ct = 1.0 / limit_scaling(std::max(mean, qn));
        for (auto& v : P.x) v *= ct;
        for (auto& v : q) v *= ct;
        c *= ct;
      }
      std::vector<double> l(m), u(m);
      for (int i = 0; i < m; ++i) {
        l[i] = (pr.l[i] <= -kInf) ? -kInf : pr.l[i] * E[i];
        u[i] = (pr.u[i] >= kInf) ? kInf : pr.u[i] * E[i];
      }
      // ---- rho vector + KKT ----
      std::vector<int> ctype(m);
      for (int i = 0; i < m; ++i) {
        if (l[i] < -kInf * kMinScaling && u[i] > kInf * kMinScaling) ctype[i] = -1;
        else if (u[i] - l[i] < kRhoTol) ctype[i] = 1;
        else ctype[i] = 0;
      }
      double rho = st->rho;
      std::vector<double> rv(m), rinv(m);
      auto set_rho = [&](double r) {
        for (int i = 0; i < m; ++i) {
          rv[i] = ctype[i] == -1 ? kRhoMin : (ctype[i] == 1 ? kRhoEqOverIneq * r : r);
          rinv[i] = 1.0 / rv[i];
        }
      };
      set_rho(rho);
      auto fill_kkt = [&]() {
        for (int j = 0; j < n; ++j) f.K.x[f.kmap_P[j]] = P.x[j] + st->sigma;
        for (size_t p = 0; p < A.x.size(); ++p) f.K.x[f.kmap_A[p]] = A.x[p];
        for (int i = 0; i < m; ++i) f.K.x[f.kmap_rho[i]] = -rinv[i];
      };
      fill_kkt();
      ldl_numeric(f);
      // ---- ADMM ----
      std::vector<double> x(n, 0.0), z(m, 0.0), y(m, 0.0), xp(n), zp(m), xt(n), zt(m);
      std::vector<double> Ax(m), Px(n), Aty(n), rhs(n + m), prm(n + m);
      auto matvecA = [&](const std::vector<double>& v, std::vector<double>& out) {
        std::fill(out.begin(), out.end(), 0.0);
        for (int j = 0; j < n; ++j)
          for (int p = A.p[j]; p < A.p[j + 1]; ++p) out[A.i[p]] += A.x[p] * v[j];
      };
      auto matvecAt = [&](const std::vector<double>& v, std::vector<double>& out) {
        for (int j = 0; j < n; ++j) {
          double s = 0.0;
          for (int p = A.p[j]; p < A.p[j + 1]; ++p) s += A.x[p] * v[A.i[p]];
          out[j] = s;
        }
      };
      int stat = -2, it = 0;
      double prim = 0, dual = 0;
      auto residuals = [&](double& eprim, double& edual) {
        matvecA(x, Ax);
        for (int j = 0; j < n; ++j) Px[j] = P.x[j] * x[j];
        matvecAt(y, Aty);
        prim = 0.0;
        double nax = 0.0, nz = 0.0;
        for (int i = 0; i < m; ++i) {
          prim = std::max(prim, fabs(Ax[i] - z[i]));
          nax = std::max(nax, fabs(Ax[i]));
          nz = std::max(nz, fabs(z[i]));
        }
        dual = 0.0;
        double npx = 0.0, naty = 0.0, nq = 0.0;
        for (int j = 0; j < n; ++j) {
          dual = std::max(dual, fabs(Px[j] + q[j] + Aty[j]));
          npx = std::max(npx, fabs(Px[j]));
          naty = std::max(naty, fabs(Aty[j]));
          nq = std::max(nq, fabs(q[j]));
        }
        eprim = std::max(nax, nz);
        edual = std::max(npx, std::max(naty, nq));
      };
      for (it = 1; it <= st->max_iter; ++it) {
        xp = x;
        zp = z;
        for (int j = 0; j < n; ++j) rhs[j] = st->sigma * xp[j] - q[j];
        for (int i = 0; i < m; ++i) rhs[n + i] = zp[i] - rinv[i] * y[i];
        for (int k = 0; k < n + m; ++k) prm[f.pinv[k]] = rhs[k];
        ldl_solve(f, prm.data());
        for (int k = 0; k < n + m; ++k) rhs[k] = prm[f.pinv[k]];
        for (int j = 0; j < n; ++j) xt[j] = rhs[j];
        for (int i = 0; i < m; ++i) zt[i] = zp[i] + rinv[i] * (rhs[n + i] - y[i]);
        for (int j = 0; j < n; ++j) x[j] = st->alpha * xt[j] + (1.0 - st->alpha) * xp[j];
        for (int i = 0; i < m; ++i) {
          const double zr = st->alpha * zt[i] + (1.0 - st->alpha) * zp[i];
          const double zn = std::min(std::max(zr + rinv[i] * y[i], l[i]), u[i]);
          y[i] += rv[i] * (zr - zn);
          z[i] = zn;
        }
        const bool chk = (it % st->check_termination) == 0;
        const bool adp = st->adaptive_rho_interval > 0 && (it % st->adaptive_rho_interval) == 0;
        if (chk || adp || it == st->max_iter) {
          double sp, sd;
          residuals(sp, sd);
          if (chk && prim <= st->eps_abs + st->eps_rel * sp &&
              dual <= st->eps_abs + st->eps_rel * sd) {
            stat = 1;
            break;
          }
          if (adp) {
            double rn = rho * sqrt((prim / (sp + kDivTol)) / (dual / (sd + kDivTol) + kDivTol));
            rn = std::min(std::max(rn, kRhoMin), kRhoMax);
            if (rn > rho * st->adaptive_rho_tolerance || rn < rho / st->adaptive_rho_tolerance) {
              rho = rn;
              set_rho(rho);
              fill_kkt();
              ldl_numeric(f);
            }
          }
        }
      }
      if (it > st->max_iter) it = st->max_iter;
      // unscale: x = D x, y = E y / c ; CasADi: lam_x = y[:n], lam_a = y[n:]
      double* w = w_out + (size_t)b * n;
      for (int j = 0; j < n; ++j) w[j] = D[j] * x[j];
      if (lam_x_out && lam_a_out) {
        for (int j = 0; j < n; ++j) lam_x_out[(size_t)b * n + j] = E[j] * y[j] / c;
        for (int i = n; i < m; ++i) lam_a_out[(size_t)b * (m - n) + (i - n)] = E[i] * y[i] / c;
      }
      status[b] = stat;
      iters[b] = it;
    }
  }
  return 0;
}

}  // extern "C"
