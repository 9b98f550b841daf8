// The hyper-parameter fit's driver on the host, native: optimize_hyperparams_mll
// (numba_kernels.py:238-321) calls scipy.optimize.minimize(objective, x0, method="Powell",
// bounds=[(1e-5, None)] * 2 n_obj, options={xtol, ftol, maxiter}) (:305-315).  scipy's Powell is
// pure Python: ~25-35 us of interpreter work per evaluation around each device MLL call (a C3 fit
// makes ~200 evaluations), more than the device work the fit needs.  This file restates the
// algorithm of scipy 1.15 (scipy/optimize/_optimize.py: _minimize_powell, _linesearch_powell,
// _line_for_search, _minimize_scalar_bounded) operation for operation in IEEE binary64, so that
// the evaluation sequence, the evaluation count and the result are scipy's.  tan/atan (the
// one-sided line search's transform) come from a caller callback when given -- the Python mirror
// passes numpy's, which differ from the C library's in the last bit for ~0.5 % of arguments (numpy
// uses SIMD implementations), so that the evaluation points are scipy's bit for bit -- else from
// the C library (tests/test_powell.py, tests/test_gpu_fit.py compare the drivers).
//
//   bo_powell_minimize             the driver over a caller objective (a C callback)
//   bo_optimize_hyperparams_mll    the whole fit: Powell over the device MLL terms, memoised per
//                                  objective (each term depends on (x, y, pm, ls_o) only; the
//                                  correlation matrix K / pv is pv-free, numba_kernels.py:195-198)

#include "bo_common.h"

#include <math.h>
#include <string.h>

#include <unordered_map>
#include <vector>

#pragma clang fp contract(off)   // numpy evaluates every operation separately: no fused multiply-add

namespace {

struct Abort {
  int status;
};
struct MaxFun {};

struct Fn {
  bo_objective_fn fn;
  void* user;
  int n;
  bo_trig_fn trig = nullptr;    // tan (which 0) / atan (which 1); NULL = the C library
  double tan_(double x) const { return trig ? trig(x, 0) : tan(x); }
  double atan_(double x) const { return trig ? trig(x, 1) : atan(x); }
  long long nfev = 0;
  double maxfun;   // scipy's maxfun (np.inf when only maxiter is given)
  double operator()(const double* x) {
    if ((double)nfev >= maxfun) throw MaxFun{};
    ++nfev;
    double f = 0.0;
    const int st = fn(x, n, &f, user);
    if (st != BO_OK) throw Abort{st};
    return f;
  }
};

typedef std::vector<double> Vec;

bool any_nonzero(const Vec& v) {
  for (double a : v)
    if (a != 0.0) return true;   // NaN counts as non-zero (np.any)
  return false;
}

// _line_for_search: the bounds on l with lower <= x0 + alpha l <= upper; (0, 0) when empty
void line_for_search(const Vec& x0, const Vec& alpha, const Vec& lb, const Vec& ub, double& lmin,
                     double& lmax) {
  bool any = false;
  double mn = 0.0, mx = 0.0;
  bool nan_min = false, nan_max = false;
  for (size_t i = 0; i < x0.size(); ++i) {
    if (!(alpha[i] != 0.0)) continue;                       // alpha.nonzero()
    const double low = (lb[i] - x0[i]) / alpha[i];
    const double high = (ub[i] - x0[i]) / alpha[i];
    const bool pos = alpha[i] > 0;
    const double lo_i = (pos ? low : 0.0) + (pos ? 0.0 : high);
    const double hi_i = (pos ? high : 0.0) + (pos ? 0.0 : low);
    if (!any) {
      mn = lo_i;
      mx = hi_i;
      any = true;
    } else {
      if (lo_i > mn) mn = lo_i;
      if (hi_i < mx) mx = hi_i;
    }
    nan_min = nan_min || lo_i != lo_i;                       // np.max / np.min propagate NaN
    nan_max = nan_max || hi_i != hi_i;
  }
  if (!any) throw Abort{BO_ERR_ARG};                         // np.max of an empty array raises
  if (nan_min) mn = NAN;
  if (nan_max) mx = NAN;
  if (mx >= mn) {
    lmin = mn;
    lmax = mx;
  } else {
    lmin = 0.0;
    lmax = 0.0;
  }
}

double sign(double v) { return v > 0 ? 1.0 : (v < 0 ? -1.0 : (v == 0 ? 0.0 : v)); }   // np.sign

// _minimize_scalar_bounded (fminbound): Brent's bounded minimiser of f on [x1, x2]
template <class F>
void scalar_bounded(F&& func, double x1, double x2, double xatol, double& xbest, double& fbest) {
  const int maxfun = 500;
  if (!isfinite(x1) || !isfinite(x2) || x1 > x2) throw Abort{BO_ERR_ARG};
  const double sqrt_eps = sqrt(2.2e-16);
  const double golden_mean = 0.5 * (3.0 - sqrt(5.0));
  double a = x1, b = x2;
  double fulc = a + golden_mean * (b - a);
  double nfc = fulc, xf = fulc;
  double rat = 0.0, e = 0.0;
  double x = xf;
  double fx = func(x);
  int num = 1;
  double fu = INFINITY;
  double ffulc = fx, fnfc = fx;
  double xm = 0.5 * (a + b);
  double tol1 = sqrt_eps * fabs(xf) + xatol / 3.0;
  double tol2 = 2.0 * tol1;
  while (fabs(xf - xm) > (tol2 - 0.5 * (b - a))) {
    bool golden = true;
    if (fabs(e) > tol1) {                                     // parabolic fit
      golden = false;
      double r = (xf - nfc) * (fx - ffulc);
      double q = (xf - fulc) * (fx - fnfc);
      double p = (xf - fulc) * q - (xf - nfc) * r;
      q = 2.0 * (q - r);
      if (q > 0.0) p = -p;
      q = fabs(q);
      r = e;
      e = rat;
      if ((fabs(p) < fabs(0.5 * q * r)) && (p > q * (a - xf)) && (p < q * (b - xf))) {
        rat = (p + 0.0) / q;
        x = xf + rat;
        if (((x - a) < tol2) || ((b - x) < tol2)) {
          const double si = sign(xm - xf) + ((xm - xf) == 0 ? 1.0 : 0.0);
          rat = tol1 * si;
        }
      } else {
        golden = true;
      }
    }
    if (golden) {                                             // golden-section step
      e = xf >= xm ? a - xf : b - xf;
      rat = golden_mean * e;
    }
    const double si = sign(rat) + (rat == 0 ? 1.0 : 0.0);
    const double ar = fabs(rat);
    const double step = (ar != ar || tol1 != tol1) ? NAN : (ar > tol1 ? ar : tol1);   // np.maximum
    x = xf + si * step;
    fu = func(x);
    num += 1;
    if (fu <= fx) {
      if (x >= xf) a = xf;
      else b = xf;
      fulc = nfc; ffulc = fnfc;
      nfc = xf; fnfc = fx;
      xf = x; fx = fu;
    } else {
      if (x < xf) a = x;
      else b = x;
      if ((fu <= fnfc) || (nfc == xf)) {
        fulc = nfc; ffulc = fnfc;
        nfc = x; fnfc = fu;
      } else if ((fu <= ffulc) || (fulc == xf) || (fulc == nfc)) {
        fulc = x; ffulc = fu;
      }
    }
    xm = 0.5 * (a + b);
    tol1 = sqrt_eps * fabs(xf) + xatol / 3.0;
    tol2 = 2.0 * tol1;
    if (num >= maxfun) break;
  }
  xbest = xf;
  fbest = fx;
}

// _linesearch_powell with bounds: minimise func(p + alpha xi); returns (fret, p + xi', xi')
void linesearch(Fn& func, Vec& p, Vec& xi, double tol, const Vec& lb, const Vec& ub, double& fval) {
  const size_t n = p.size();
  if (!any_nonzero(xi)) return;                               // (fval, p, xi) unchanged
  double b0, b1;
  line_for_search(p, xi, lb, ub, b0, b1);
  Vec pt(n);
  auto myfunc = [&](double alpha) {
    for (size_t i = 0; i < n; ++i) pt[i] = p[i] + alpha * xi[i];
    return func(pt.data());
  };
  const bool ninf0 = isinf(b0) && b0 < 0, pinf1 = isinf(b1) && b1 > 0;
  double xs, fs, alpha;
  if (ninf0 && pinf1) {
    throw Abort{BO_ERR_UNSUPPORTED};                          // unbounded line (Brent + bracket): not needed by the fit's bounds
  } else if (!ninf0 && !pinf1) {
    scalar_bounded(myfunc, b0, b1, tol / 100, xs, fs);
    alpha = xs;
  } else {
    // one-sided: the tangent maps (-pi/2, pi/2) onto the line
    scalar_bounded([&](double t) { return myfunc(func.tan_(t)); }, func.atan_(b0), func.atan_(b1), tol / 100, xs,
                   fs);
    alpha = func.tan_(xs);
  }
  for (size_t i = 0; i < n; ++i) {
    xi[i] = alpha * xi[i];
    p[i] = p[i] + xi[i];
  }
  fval = fs;
}

int powell(Fn& func, Vec& x, const Vec& lb, const Vec& ub, double xtol, double ftol, double maxiter,
           std::vector<Vec>& direc, bo_powell_result* res) {
  const int N = (int)x.size();
  long long iter = 0;
  double fval = 0.0;
  try {
    fval = func(x.data());
    Vec x1 = x;
    while (true) {
      const double fx = fval;
      int bigind = 0;
      double delta = 0.0;
      for (int i = 0; i < N; ++i) {
        Vec direc1 = direc[i];
        const double fx2 = fval;
        linesearch(func, x, direc1, xtol * 100, lb, ub, fval);
        if ((fx2 - fval) > delta) {
          delta = fx2 - fval;
          bigind = i;
        }
      }
      iter += 1;
      const double bnd = ftol * (fabs(fx) + fabs(fval)) + 1e-20;
      if (2.0 * (fx - fval) <= bnd) break;
      if ((double)func.nfev >= func.maxfun) break;
      if ((double)iter >= maxiter) break;
      if (isnan(fx) && isnan(fval)) break;
      // the extrapolated point, kept inside the bounds
      Vec direc1(N);
      for (int i = 0; i < N; ++i) direc1[i] = x[i] - x1[i];
      x1 = x;
      double lmin, lmax;
      line_for_search(x, direc1, lb, ub, lmin, lmax);
      const double m = (1.0 < lmax) ? 1.0 : lmax;             // Python min(lmax, 1)
      Vec x2(N);
      for (int i = 0; i < N; ++i) x2[i] = x[i] + m * direc1[i];
      const double fx2 = func(x2.data());
      if (fx > fx2) {
        double t = 2.0 * (fx + fx2 - 2.0 * fval);
        double temp = (fx - fval - delta);
        t *= temp * temp;
        temp = fx - fx2;
        t -= delta * temp * temp;
        if (t < 0.0) {
          linesearch(func, x, direc1, xtol * 100, lb, ub, fval);
          if (any_nonzero(direc1)) {
            direc[bigind] = direc[N - 1];
            direc[N - 1] = direc1;
          }
        }
      }
    }
  } catch (const MaxFun&) {
  } catch (const Abort& a) {
    return a.status;
  }
  int warn = 0;
  bool oob = false, xnan = false;
  for (int i = 0; i < N; ++i) {
    oob = oob || lb[i] > x[i] || x[i] > ub[i];
    xnan = xnan || isnan(x[i]);
  }
  if (oob) warn = 4;
  else if ((double)func.nfev >= func.maxfun) warn = 1;
  else if ((double)iter >= maxiter) warn = 2;
  else if (isnan(fval) || xnan) warn = 3;
  res->fun = fval;
  res->nfev = func.nfev;
  res->nit = iter;
  res->warnflag = warn;
  return BO_OK;
}

// ----------------------------------------------------------------- the MLL objective
struct MllCtx {
  const double* x;
  int dim;
  const double* y;
  long long ld_y;
  double* km;
  long long ld;
  int n_obj;
  const double* pm;
  long long n;
  double jitter;
  void* ws;
  size_t ws_bytes;
  void* stream;
  std::unordered_map<unsigned long long, double> cache[BO_MAX_OBJ];
  double last[2 * BO_MAX_OBJ];
  bool have_last = false;
  long long device_calls = 0;
};

unsigned long long key_of(double v) {
  v = v + 0.0;                                                // -0.0 and 0.0 are one key (Python float)
  unsigned long long b;
  memcpy(&b, &v, 8);
  return b;
}

// -sum_o mll_o(ls_o) (numba_kernels.py:274-288): every term once per distinct ls_o (NaN never
// memoised: NaN != NaN as a dict key), one device call over the objectives whose ls changed
// (all of them when more than one changed), summed in objective order like np.sum (:235)
int mll_objective(const double* p, int32_t n, double* f, void* user) {
  MllCtx& c = *(MllCtx*)user;
  const int no = c.n_obj;
  if (n != 2 * no) return BO_ERR_ARG;
  memcpy(c.last, p, sizeof(double) * n);
  c.have_last = true;
  const double* ls = p;
  const double* pv = p + no;
  int todo[BO_MAX_OBJ], nt = 0;
  for (int o = 0; o < no; ++o)
    if (ls[o] != ls[o] || !c.cache[o].count(key_of(ls[o]))) todo[nt++] = o;
  double nan_term[BO_MAX_OBJ];
  if (nt) {
    const int o0 = nt == 1 ? todo[0] : 0, cnt = nt == 1 ? 1 : no;
    double terms[BO_MAX_OBJ];
    const int st = bo_compute_mll_each_jitter(terms, c.x, c.dim, c.y + o0, c.ld_y, c.km + (long long)o0 * c.ld * c.ld,
                                              c.ld, cnt, c.pm + o0, pv + o0, ls + o0, c.n, c.jitter, c.ws,
                                              c.ws_bytes, c.stream);
    c.device_calls += 1;
    if (st != BO_OK) return st;
    for (int i = 0; i < cnt; ++i) {
      const int o = o0 + i;
      if (ls[o] != ls[o]) nan_term[o] = terms[i];
      else c.cache[o][key_of(ls[o])] = terms[i];
    }
  }
  double tot = 0.0;
  for (int o = 0; o < no; ++o) tot += ls[o] != ls[o] ? nan_term[o] : c.cache[o][key_of(ls[o])];
  *f = -tot;
  return BO_OK;
}

}  // namespace

extern "C" {

int bo_powell_minimize(bo_objective_fn fn, void* user, double* x, int32_t n, const double* lb,
                       const double* ub, double xtol, double ftol, int64_t maxiter, int64_t maxfev,
                       bo_trig_fn trig, double* direc, bo_powell_result* res) {
  if (!fn || !x || n < 1 || !lb || !ub || !res) return BO_ERR_ARG;
  memset(res, 0, sizeof(*res));
  // scipy's defaults: maxiter / maxfev None -> N * 1000 each; one given -> the other np.inf
  double mi = maxiter < 0 ? -1.0 : (double)maxiter, mf = maxfev < 0 ? -1.0 : (double)maxfev;
  if (mi < 0 && mf < 0) {
    mi = 1000.0 * n;
    mf = 1000.0 * n;
  } else if (mi < 0) {
    mi = INFINITY;
  } else if (mf < 0) {
    mf = INFINITY;
  }
  Fn func{fn, user, n};
  func.trig = trig;
  func.maxfun = mf;
  Vec xv(x, x + n), l(lb, lb + n), u(ub, ub + n);
  std::vector<Vec> dir(n, Vec(n, 0.0));
  for (int i = 0; i < n; ++i) dir[i][i] = 1.0;
  const int st = powell(func, xv, l, u, xtol, ftol, mi, dir, res);
  res->nfev = func.nfev;
  if (st != BO_OK) return st;
  memcpy(x, xv.data(), sizeof(double) * n);
  if (direc)
    for (int i = 0; i < n; ++i) memcpy(direc + (size_t)i * n, dir[i].data(), sizeof(double) * n);
  return BO_OK;
}

int bo_optimize_hyperparams_mll(const double* x, int32_t dim, const double* y, int64_t ld_y,
                                double* kernel_matrix, int64_t ld, int32_t n_obj, const double* prior_mean,
                                double* prior_variance, double* length_scales, int64_t n, double jitter,
                                double xtol, double ftol, int64_t maxiter, double min_bound, bo_trig_fn trig,
                                void* workspace, size_t workspace_bytes, void* stream, bo_powell_result* res,
                                double* direc) {
  if (!x || !y || !kernel_matrix || !prior_mean || !prior_variance || !length_scales || !res ||
      n_obj < 1 || n_obj > BO_MAX_OBJ || n < 1 || ld < n || dim < 1)
    return BO_ERR_ARG;
  MllCtx* c = new MllCtx();
  c->x = x; c->dim = dim; c->y = y; c->ld_y = ld_y; c->km = kernel_matrix; c->ld = ld; c->n_obj = n_obj;
  c->pm = prior_mean; c->n = n; c->jitter = jitter; c->ws = workspace; c->ws_bytes = workspace_bytes;
  c->stream = stream;
  const int np_ = 2 * n_obj;
  double x0[2 * BO_MAX_OBJ], lb[2 * BO_MAX_OBJ], ub[2 * BO_MAX_OBJ];
  for (int o = 0; o < n_obj; ++o) {          // initial guess [ls..., pv...] (:268)
    x0[o] = length_scales[o];
    x0[n_obj + o] = prior_variance[o];
  }
  for (int i = 0; i < np_; ++i) {            // bounds (HYPERPARAM_MIN_BOUND, None) (:271)
    lb[i] = min_bound;
    ub[i] = INFINITY;
  }
  int st = bo_powell_minimize(mll_objective, c, x0, np_, lb, ub, xtol, ftol, maxiter, -1, trig, direc, res);
  res->device_calls = c->device_calls;
  // compute_mll's side effect: kernel_matrix holds the Gram of the last evaluated hyper-parameters
  if (c->have_last && (st == BO_OK || st == BO_ERR_NOT_PD)) {
    const int st2 = bo_update_k(kernel_matrix, ld, n_obj, x, dim, 0, n, c->last + n_obj, c->last, stream);
    if (st == BO_OK) st = st2;
  }
  delete c;
  if (st != BO_OK) return st;
  for (int o = 0; o < n_obj; ++o) {          // in place (:318-319)
    length_scales[o] = x0[o];
    prior_variance[o] = x0[n_obj + o];
  }
  return BO_OK;
}

}  // extern "C"
