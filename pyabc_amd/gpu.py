"""Torch-plumbing wrappers over the libabcgpu C ABI.

PyTorch is used only to own device memory and to name the HIP stream; every
computation below is a hand-written HIP kernel reached through
``pyabc_amd._native``.  All tensors are float64 / int64 on the current
device unless stated.
"""
import math

import numpy as np

from . import _native as nat

try:
    import torch
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None

F64 = None if torch is None else torch.float64
I64 = None if torch is None else torch.int64


class NoDeviceError(RuntimeError):
    pass


_have_device = False


def require_device():
    """The GPU path needs a HIP device and the native library: fail loudly.
    (The availability check runs once: it reads the environment each time.)"""
    global _have_device
    if not _have_device:
        if torch is None or not torch.cuda.is_available():
            raise NoDeviceError("pyabc_amd GPU path needs an MI355X (HIP device)")
        nat.load()
        _have_device = True
    return torch.device("cuda", torch.cuda.current_device())


def stream_ptr():
    """Raw hipStream_t of the current torch stream (fast C-level query)."""
    return torch._C._cuda_getCurrentRawStream(torch.cuda.current_device())


def p(t):
    """Raw device pointer of a contiguous tensor (or None)."""
    if t is None:
        return None
    assert t.is_contiguous(), "kernels take contiguous tensors"
    return t.data_ptr()


_ws = {}


def workspace(nbytes, slot="main"):
    """A cached device scratch buffer of at least nbytes (per device/slot)."""
    dev = torch.cuda.current_device()
    key = (dev, slot)
    buf = _ws.get(key)
    nbytes = max(int(nbytes), 256)
    if buf is None or buf.numel() < nbytes:
        # zero-filled once: abc_candidates_round's tile ticket counter and
        # abc_weighted_quantile's control block live in their slots' first
        # bytes, and every call leaves them zero
        buf = torch.zeros(int(nbytes * 1.25) + 256, dtype=torch.uint8,
                          device=f"cuda:{dev}")
        _ws[key] = buf
    return buf


class HostFuture:
    """Device -> pinned host copy enqueued on the current stream; .get()
    waits for that copy only (no device-wide sync), so the host can keep
    queueing work while the value is produced."""

    # events are reused once waited on: a torch.cuda.Event creates its HIP
    # event at its first record (~35 us of host time, several per generation)
    _events = {}

    def __init__(self, t, _record=True):
        self._h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        self._h.copy_(t, non_blocking=True)
        self._dev = t.device.index if t.is_cuda else torch.cuda.current_device()
        self._pooled = _record
        self._ev = None
        if _record:
            pool = HostFuture._events.setdefault(self._dev, [])
            self._ev = pool.pop() if pool else torch.cuda.Event()
            self._ev.record(torch.cuda.current_stream(self._dev))
        self._v = None

    @classmethod
    def group(cls, ts):
        """Futures of several tensors behind one event record (each record
        costs ~30 us of host time on this stack)."""
        futs = [cls(t, _record=False) for t in ts]
        if futs:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(futs[-1]._dev))
            for f in futs:
                f._ev = ev
        return futs

    def get(self):
        if self._v is None:
            self._ev.synchronize()
            self._v = self._h.numpy().copy()
            pool = HostFuture._events.setdefault(self._dev, [])
            if self._pooled and len(pool) < 64:
                pool.append(self._ev)
            self._h = self._ev = None
        return self._v

    def __deepcopy__(self, memo):
        return self          # the value is immutable once produced

    def __getstate__(self):
        return {"_v": self.get(), "_h": None, "_ev": None}


_flat = {}


def flat_prior(d, device):
    """Device (kind, params) of a flat prior over d parameters (cached):
    the proposal kernels' "no prior" arguments for a plain Transition.rvs."""
    key = (int(d), str(device))
    if key not in _flat:
        _flat[key] = (as_dev(np.full(d, -1), dtype=torch.int32, device=device),
                      torch.zeros(4 * d, dtype=F64, device=device))
    return _flat[key]


def as_dev(a, dtype=None, device=None):
    """numpy / list / tensor -> contiguous device tensor."""
    dtype = dtype or F64
    device = device or require_device()
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype,
                           device=device).contiguous()


# ---- reductions -----------------------------------------------------------

def weighted_moments(X, w, with_max=False):
    """(sum w, sum w^2, mean [d], cov_biased [d, d]) as float64 numpy
    (+ max w with with_max), one device-to-host read."""
    N, d = X.shape
    out = torch.empty(3 + d + d * d, dtype=F64, device=X.device)
    nb = nat.query("abc_weighted_moments_workspace", N, d)
    ws = workspace(nb)
    nat.call("abc_weighted_moments", p(X), p(w), N, d, p(out), p(ws), ws.numel(),
             stream_ptr())
    o = out.cpu().numpy()
    res = (o[0], o[1], o[2:2 + d].copy(), o[2 + d:2 + d + d * d].reshape(d, d).copy())
    return res + (o[2 + d + d * d],) if with_max else res


def inclusive_scan(x, out=None):
    n = x.numel()
    out = torch.empty_like(x) if out is None else out
    nb = nat.query("abc_scan_workspace", n)
    ws = workspace(nb, "scan")
    nat.call("abc_inclusive_scan_f64", p(x), p(out), n, p(ws), ws.numel(),
             stream_ptr())
    return out


def normalize_weights(w):
    """In-place w /= sum(w); returns device stats [sum, ESS, sum w^2]."""
    n = w.numel()
    stats = torch.empty(3, dtype=F64, device=w.device)
    nb = nat.query("abc_normalize_weights_workspace", n)
    ws = workspace(nb, "norm")
    nat.call("abc_normalize_weights", p(w), n, p(stats), p(ws), ws.numel(),
             stream_ptr())
    return stats


# ---- MultivariateNormalTransition -----------------------------------------

def mvn_pack(X, w, mu, U, shift, prec, with_range=False, shift_dev=None):
    """Population operand image; with_range also returns the device range
    [max |y_jk|, max |y_j|^2 / 2] (log2-scaled whitened units).  shift_dev:
    a device scalar read instead of the host shift (X3 only)."""
    N, d = X.shape
    r = U.shape[1]
    nb = nat.query("abc_mvn_packed_bytes", N, r, prec)
    packed = torch.empty(nb, dtype=torch.uint8, device=X.device)
    rng = torch.empty(2, dtype=F64, device=X.device) if with_range else None
    nat.call("abc_mvn_pack_population", p(X), p(w), N, d, p(mu), p(U), r,
             float(shift), p(shift_dev), prec, p(packed), p(rng), stream_ptr())
    return (packed, rng) if with_range else packed


def weighted_moments_dev(X, w):
    """abc_weighted_moments' output left on the device: [sum w, sum w^2,
    mean (d), biased cov (d x d), max w]."""
    N, d = X.shape
    out = torch.empty(3 + d + d * d, dtype=F64, device=X.device)
    nb = nat.query("abc_weighted_moments_workspace", N, d)
    ws = workspace(nb)
    nat.call("abc_weighted_moments", p(X), p(w), N, d, p(out), p(ws), ws.numel(),
             stream_ptr())
    return out


def mvn_fit(moments, d, scaling, bw_rule):
    """abc_mvn_fit: (cov, evec, evals, U, L, stats) as device tensors, from
    weighted_moments_dev's output; no host read."""
    dev = moments.device
    blob = torch.empty(4 * d * d + d + 8, dtype=F64, device=dev)
    cov, evec, U, L = (blob[k * d * d:(k + 1) * d * d].view(d, d) for k in range(4))
    evals = blob[4 * d * d:4 * d * d + d]
    stats = blob[4 * d * d + d:]
    nat.call("abc_mvn_fit", p(moments), d, float(scaling), int(bw_rule), p(cov), p(evec),
             p(evals), p(U), p(L), p(stats), stream_ptr())
    return cov, evec, evals, U, L, stats


def mvn_logpdf(x, packed, N, mu, U, prec, log_const, out=None, X=None, w=None,
               shift=0.0, hint=None):
    """hint: optional device int64 [M] population rows near the candidates
    (the proposal's ancestors; X3 skips its max pre-pass)."""
    M, d = x.shape
    r = U.shape[1]
    out = torch.empty(M, dtype=F64, device=x.device) if out is None else out
    if M == 0:
        return out
    if hint is not None:
        if hint.dtype != I64 or hint.numel() != M:
            raise ValueError("mvn_logpdf: hint must be int64 [M]")
        hint = hint.contiguous()
    nb = nat.query("abc_mvn_logpdf_workspace", M, N, r, prec)
    ws = workspace(nb, "mvn")
    nat.call("abc_mvn_logpdf", p(x), M, d, p(packed), p(X), p(w), N, p(mu),
             p(U), r, prec, float(log_const), float(shift), p(out), p(hint),
             p(ws), ws.numel(), stream_ptr())
    return out


def mvn_x3_layout(r):
    """(kernel, K slots per pair, candidate tiles per wave) the x3 density
    runs at whitened rank r (kernel 0 = mvn_x3_kernel<K / 32, tiles>)."""
    import ctypes
    k, ct = ctypes.c_int(0), ctypes.c_int(0)
    kernel = int(nat.load().abc_mvn_x3_layout(int(r), ctypes.byref(k), ctypes.byref(ct)))
    return kernel, int(k.value), int(ct.value)


def mvn_logpdf_direct(x, X, w, U, V, support_tol, log_const, out=None):
    M, d = x.shape
    N = X.shape[0]
    r = 0 if U is None else U.shape[1]
    nv = 0 if V is None else V.shape[1]
    out = torch.empty(M, dtype=F64, device=x.device) if out is None else out
    if M == 0:
        return out
    nat.call("abc_mvn_logpdf_direct", p(x), M, p(X), p(w), N, d,
             p(U) if r else None, r, p(V) if nv else None, nv,
             float(support_tol), float(log_const), p(out), stream_ptr())
    return out


# ---- proposal / prior / simulator / distance / acceptance ----------------

def cdf_guide(cdf):
    """int32 guide table of an inclusive weight scan (abc_cdf_guide)."""
    N = cdf.numel()
    guide = torch.empty(N, dtype=torch.int32, device=cdf.device)
    nat.call("abc_cdf_guide", p(cdf), N, p(guide), stream_ptr())
    return guide


def ancestor_table(X, cdf):
    """Ancestor table of a population (abc_ancestor_table): padded row
    records with their scan value + exact-bin guide, for the fused rounds."""
    N, d = X.shape
    nb = nat.query("abc_ancestor_table_bytes", int(N), int(d))
    t = torch.empty(int(nb), dtype=torch.uint8, device=X.device)
    if t.data_ptr() % 128:
        raise RuntimeError("ancestor_table: allocation not 128-byte aligned")
    nat.call("abc_ancestor_table", p(X), p(cdf), int(N), int(d), p(t), t.numel(),
             stream_ptr())
    return t


def propose(X, cdf, L, prior_kind, prior_params, seed, generation, idx0, B,
            max_attempts, d, per_particle_L=False, guide=None):
    dev = prior_params.device
    theta = torch.empty((B, d), dtype=F64, device=dev)
    lp = torch.empty(B, dtype=F64, device=dev)
    anc = torch.empty(B, dtype=I64, device=dev)
    att = torch.empty(B, dtype=torch.int32, device=dev)
    N = 0 if X is None else X.shape[0]
    fn = "abc_local_propose" if per_particle_L else "abc_propose"
    nat.call(fn, p(X), p(cdf), p(guide), N, d, p(L), p(prior_kind), p(prior_params),
             int(seed) & (2 ** 64 - 1), int(generation) & 0xFFFFFFFF, int(idx0),
             int(B), int(max_attempts), p(theta), p(lp), p(anc), p(att),
             stream_ptr())
    return theta, lp, anc, att


def prior_logpdf(theta, prior_kind, prior_params, out=None):
    B, d = theta.shape
    out = torch.empty(B, dtype=F64, device=theta.device) if out is None else out
    nat.call("abc_prior_logpdf", p(theta), B, d, p(prior_kind), p(prior_params),
             p(out), stream_ptr())
    return out


def simulate_linear_gaussian(theta, src, a, sigma, seed, generation, idx0,
                             out=None):
    B, d = theta.shape
    S = src.numel()
    out = torch.empty((B, S), dtype=F64, device=theta.device) if out is None else out
    nat.call("abc_simulate_linear_gaussian", p(theta), B, d, S, p(src), p(a),
             p(sigma), int(seed) & (2 ** 64 - 1), int(generation) & 0xFFFFFFFF,
             int(idx0), p(out), stream_ptr())
    return out


def pnorm(x, x0, wf, pval, out=None):
    B, S = x.shape
    out = torch.empty(B, dtype=F64, device=x.device) if out is None else out
    nat.call("abc_pnorm", p(x), B, S, p(x0), p(wf), float(pval), p(out),
             stream_ptr())
    return out


def pnorm_accept(x, x0, wf, pval, eps, cap, att=None, max_attempts=0):
    """Accept tail of one staged round (abc_pnorm_accept): the positions of
    the first `cap` rows of x [B, S] whose p-norm distance to x0 is <= eps
    (and whose proposal did not give up), and the number accepted [1] int64,
    without a distance array.  x must be contiguous float64."""
    B, S = x.shape
    if x.dtype != F64 or not x.is_contiguous():
        x = x.to(F64).contiguous()
    cap = int(min(max(cap, 0), B))
    idx = torch.empty(max(cap, 1), dtype=I64, device=x.device)
    cnt = torch.empty(1, dtype=I64, device=x.device)
    nb = nat.query("abc_candidates_workspace", int(B))
    ws = workspace(nb, "candidates")
    nat.call("abc_pnorm_accept", p(x), int(B), int(S), p(x0), p(wf), float(pval),
             float(eps), p(att), int(max_attempts), cap, p(idx), p(cnt), p(ws),
             ws.numel(), stream_ptr())
    return idx, cnt


def prior_uniforms(att, k, seed, generation, idx0, B=None):
    """Uniforms in (0, 1) of the candidates' prior streams for dimension k
    (abc_prior_uniforms): the source of an ABC_PRIOR_HOST coordinate's draw."""
    B = att.numel() if B is None else B
    dev = att.device if att is not None else require_device()
    u = torch.empty(B, dtype=F64, device=dev)
    nat.call("abc_prior_uniforms", p(att) if att is not None else None, p(u), B, int(k),
             int(seed) & 0xFFFFFFFFFFFFFFFF, int(generation) & 0xFFFFFFFF, int(idx0),
             stream_ptr())
    return u


def mask_gave_up(dist, att, max_attempts, value=float("nan")):
    """dist[b] = value where att[b] > max_attempts (in place); NaN (never
    accepted, even at eps = inf) unless the caller passes the zero-probability
    density of a StochasticAcceptor."""
    nat.call("abc_mask_gave_up", p(dist), p(att), dist.numel(), int(max_attempts),
             float(value), stream_ptr())
    return dist


def accept_compact(d, eps, idx_out=None, count_out=None):
    B = d.numel()
    idx = torch.empty(max(B, 1), dtype=I64, device=d.device) if idx_out is None else idx_out
    cnt = torch.empty(1, dtype=I64, device=d.device) if count_out is None else count_out
    nb = nat.query("abc_compact_workspace", B)
    ws = workspace(nb, "compact")
    nat.call("abc_accept_compact", p(d), B, float(eps), p(idx), p(cnt), p(ws),
             ws.numel(), stream_ptr())
    return idx, cnt


class CandidateRound:
    """The device description of one generation's candidate closure for the
    fused kernels (abc_candidate_spec): proposal (MVN / LocalTransition
    arrays, or X=None for the prior), LinearGaussianModel (src, a, sigma),
    PNormDistance (x0, wf, p).  Holds the tensors the struct points to."""

    def __init__(self, d, S, prior_kind, prior_params, src, a, sigma, x0, wf,
                 p, seed, generation, max_attempts, X=None, cdf=None,
                 guide=None, L=None, per_particle_L=False, anc_table=None):
        self._keep = [t for t in (prior_kind, prior_params, src, a, sigma, x0,
                                  wf, X, cdf, guide, L, anc_table) if t is not None]
        for t in self._keep:
            assert t.is_contiguous() and t.is_cuda
        if src.dtype != torch.int32 or prior_kind.dtype != torch.int32:
            raise TypeError("CandidateRound: src / prior_kind must be int32")
        self.d, self.S = int(d), int(S)
        self.spec = nat.CandidateSpec()
        s = self.spec
        s.d, s.S = self.d, self.S
        s.X, s.cdf, s.guide = _ptr(X), _ptr(cdf), _ptr(guide)
        s.N = 0 if X is None else int(X.shape[0])
        s.L, s.per_particle_L = _ptr(L), int(bool(per_particle_L))
        s.prior_kind, s.prior_params = _ptr(prior_kind), _ptr(prior_params)
        s.max_attempts = int(max_attempts)
        s.src, s.a, s.sigma = _ptr(src), _ptr(a), _ptr(sigma)
        s.x0, s.wf, s.p = _ptr(x0), _ptr(wf), float(p)
        s.seed = int(seed) & (2 ** 64 - 1)
        s.generation = int(generation) & 0xFFFFFFFF
        if X is not None and anc_table is None:
            anc_table = ancestor_table(X, cdf)
            self._keep.append(anc_table)
        s.anc_table = _ptr(anc_table) if X is not None else None
        # the prior's support box, once per generation (not per round)
        self._box = torch.empty(2 * self.d, dtype=F64, device=prior_params.device)
        nat.call("abc_prior_support_box", _ptr(prior_kind), _ptr(prior_params), self.d,
                 _ptr(self._box), stream_ptr())
        s.support_box = _ptr(self._box)
        self.device = prior_params.device

    def run(self, idx0, B, eps, cap, filter=True, rec_x=None, idx_out=None,
            count_out=None, eps_dev=None, eps_scale=1.0):
        """One round (abc_candidates_round): (idx [cap] int64 positions of the
        first cap accepted, count [1] int64 accepted in the round).  eps_dev
        (device scalar, optional): the threshold is eps_dev * eps_scale, read
        on the device."""
        import ctypes as C
        idx = (torch.empty(max(int(cap), 1), dtype=I64, device=self.device)
               if idx_out is None else idx_out)
        cnt = (torch.empty(1, dtype=I64, device=self.device)
               if count_out is None else count_out)
        if rec_x is not None and tuple(rec_x.shape) != (int(B), self.S):
            raise ValueError("CandidateRound.run: rec_x must be [B, S]")
        nb = nat.query("abc_candidates_workspace", int(B))
        ws = workspace(nb, "candidates")
        nat.call("abc_candidates_round", C.addressof(self.spec), int(idx0), int(B),
                 float(eps), p(eps_dev), float(eps_scale), int(bool(filter)), int(cap),
                 p(idx), p(cnt), p(rec_x),
                 p(ws), ws.numel(), stream_ptr())
        return idx, cnt

    def propose(self, idx0, B, with_lp=True):
        """Proposals of candidates idx0 .. idx0 + B - 1 only
        (abc_candidates_propose): theta [B, d], prior log-density [B] (None
        unless with_lp), ancestor [B] (int64), attempts [B] (int32) -- the
        rows gpu.propose returns, through the round's proposal (ancestor
        table, support box computed once)."""
        import ctypes as C
        dev = self.device
        B = int(B)
        theta = torch.empty((B, self.d), dtype=F64, device=dev)
        lp = torch.empty(B, dtype=F64, device=dev) if with_lp else None
        anc = torch.empty(B, dtype=I64, device=dev)
        att = torch.empty(B, dtype=torch.int32, device=dev)
        if B:
            ws = workspace(nat.query("abc_candidates_propose_workspace"), "propose")
            nat.call("abc_candidates_propose", C.addressof(self.spec), int(idx0), B,
                     p(theta), p(lp), p(anc), p(att), p(ws), ws.numel(), stream_ptr())
        return theta, lp, anc, att

    def regen(self, idx0, idx, out=None):
        """Rows of the candidates idx0 + idx[i] (abc_candidates_regen):
        theta [n, d], prior log-density [n], ancestor [n], x [n, S], dist [n];
        out: these five tensors (contiguous) to write into."""
        import ctypes as C
        n = int(idx.numel())
        dev = self.device
        if out is not None:
            theta, lp, anc, x, dist = out
            if not (tuple(theta.shape) == (n, self.d) and lp.numel() == n and anc.numel() == n
                    and tuple(x.shape) == (n, self.S) and dist.numel() == n
                    and anc.dtype == I64 and all(t.is_contiguous() for t in out)):
                raise ValueError("CandidateRound.regen: out does not match the rows")
        else:
            theta = torch.empty((n, self.d), dtype=F64, device=dev)
            lp = torch.empty(n, dtype=F64, device=dev)
            anc = torch.empty(n, dtype=I64, device=dev)
            x = torch.empty((n, self.S), dtype=F64, device=dev)
            dist = torch.empty(n, dtype=F64, device=dev)
        if n:
            nat.call("abc_candidates_regen", C.addressof(self.spec), int(idx0),
                     p(idx.contiguous()), n, None, p(theta), p(lp), p(anc), p(x), p(dist),
                     stream_ptr())
        return theta, lp, anc, x, dist

    def regen_into(self, idx0, idx_ptr, n, ptrs, n_dev=None):
        """regen into raw device addresses (theta, lp, anc, x, dist rows of
        n candidates; idx_ptr: their int64 indices) -- the sampler's pooled
        per-generation rows, whose views it builds once per generation.
        n_dev (device int64 [1]): the rows are the first min(n, n_dev[0]),
        so the launch can be queued before the host has read that count."""
        import ctypes as C
        if n:
            nat.call("abc_candidates_regen", C.addressof(self.spec), int(idx0), idx_ptr,
                     int(n), p(n_dev), *ptrs, stream_ptr())


def round_keep(counts, need, rank, out=None):
    """abc_round_keep: this rank's kept rows of a round (device int64 [1])
    from the all-gathered per-rank accept counts (device int64 [ws])."""
    out = torch.empty(1, dtype=I64, device=counts.device) if out is None else out
    nat.call("abc_round_keep", p(counts), int(counts.numel()), int(rank), int(need), p(out),
             stream_ptr())
    return out


def _ptr(t):
    return None if t is None else p(t)


def gather_rows(x, idx, n=None):
    n = idx.numel() if n is None else n
    cols = 1 if x.dim() == 1 else x.shape[1]
    out = torch.empty((n, cols) if x.dim() > 1 else (n,), dtype=F64,
                      device=x.device)
    nat.call("abc_gather_rows", p(x), p(idx), n, cols, p(out), stream_ptr())
    return out


def gather_rows_batch(arrays, idx, n=None):
    """[a[idx[:n]] for a in arrays] in one launch (8-byte dtypes; 1-D arrays
    are treated as one column)."""
    import ctypes as C
    n = idx.numel() if n is None else int(n)
    outs = [torch.empty((n,) + tuple(a.shape[1:]), dtype=a.dtype, device=a.device)
            for a in arrays]
    if n == 0:
        return outs
    k = len(arrays)
    ins_c = (C.c_void_p * k)(*[p(a) for a in arrays])
    outs_c = (C.c_void_p * k)(*[p(o) for o in outs])
    cols_c = (C.c_int * k)(*[1 if a.dim() == 1 else int(a.shape[1]) for a in arrays])
    row0_c = (C.c_int64 * k)(*([0] * k))
    nat.call("abc_gather_rows_batch", k, C.addressof(ins_c), C.addressof(cols_c),
             C.addressof(outs_c), C.addressof(row0_c), p(idx), n, stream_ptr())
    return outs


def importance_weights(prior_lp, trans_lp, scale=1.0, acc_w=None):
    A = prior_lp.numel()
    w = torch.empty(A, dtype=F64, device=prior_lp.device)
    nat.call("abc_importance_weights", p(prior_lp), p(trans_lp), p(acc_w), A,
             float(scale), p(w), stream_ptr())
    return w


# ---- sort / quantile / column statistics ---------------------------------

def sort_pairs(keys, vals):
    N = keys.numel()
    ko = torch.empty_like(keys)
    vo = torch.empty_like(vals)
    nb = nat.query("abc_sort_pairs_workspace", N)
    ws = workspace(nb, "sort")
    nat.call("abc_sort_pairs_f64", p(keys), p(vals), N, p(ko), p(vo), p(ws),
             ws.numel(), stream_ptr())
    return ko, vo


def weighted_quantile(points, w, alpha, sorted_path=False):
    """Weighted quantile on the device (weighted_statistics.py:27-43) -> q [1]
    (device).  The weighted MSD select (abc_weighted_quantile) leaves NaN when
    the knots sit in ties by the thousand; resolve_quantile reruns those on the
    sort-based kernel (sorted_path=True)."""
    N = points.numel()
    q = torch.empty(1, dtype=F64, device=points.device)
    name = "abc_weighted_quantile_sorted" if sorted_path else "abc_weighted_quantile"
    nb = nat.query(name + "_workspace", N)
    # the select's own slot: its control block stays zero between calls
    ws = workspace(nb, "sort" if sorted_path else "quantile")
    nat.call(name, p(points), p(w), N, float(alpha), p(q), p(ws), ws.numel(), stream_ptr())
    return q


def resolve_quantile(q_host, points, w, alpha):
    """The host value of a weighted_quantile result: a NaN from the select
    (undecided, not a NaN input) is recomputed on the sort-based path."""
    v = float(q_host)
    if v != v:
        v = float(weighted_quantile(points, w, alpha, sorted_path=True).cpu()[0])
    return v


def column_std(X):
    R, S = X.shape
    out = torch.empty(S, dtype=F64, device=X.device)
    nb = nat.query("abc_column_stats_workspace", R, S)
    ws = workspace(nb, "colstats")
    nat.call("abc_column_std", p(X), R, S, p(out), p(ws), ws.numel(), stream_ptr())
    return out


def column_mad(X):
    R, S = X.shape
    out = torch.empty(S, dtype=F64, device=X.device)
    nb = nat.query("abc_column_stats_workspace", R, S)
    ws = workspace(nb, "colstats")
    nat.call("abc_column_mad", p(X), R, S, p(out), p(ws), ws.numel(), stream_ptr())
    return out


def bootstrap_cv(logdens, w, scale=1.0):
    """logdens [B, N] (bootstrapped log densities at N test points), w [N]
    -> (variation [N], cv [1]) on the device (abc_bootstrap_cv)."""
    B, N = logdens.shape
    if w.numel() != N or not logdens.is_contiguous():
        raise ValueError(f"bootstrap_cv: {w.numel()} weights for {N} test "
                         "points (or non-contiguous densities)")
    var = torch.empty(N, dtype=F64, device=logdens.device)
    cv = torch.empty(1, dtype=F64, device=logdens.device)
    nb = nat.query("abc_bootstrap_cv_workspace", N)
    ws = workspace(nb, "cv")
    nat.call("abc_bootstrap_cv", p(logdens), B, N, p(w), float(scale), p(var),
             p(cv), p(ws), ws.numel(), stream_ptr())
    return var, cv


# ---- LocalTransition -------------------------------------------------------

def local_fit(X, w, k, scaling, eps):
    N, d = X.shape
    dev = X.device
    covs = torch.empty((N, d, d), dtype=F64, device=dev)
    inv = torch.empty_like(covs)
    chol = torch.empty_like(covs)
    dets = torch.empty(N, dtype=F64, device=dev)
    lnorm = torch.empty(N, dtype=F64, device=dev)
    nb = nat.query("abc_local_fit_workspace", N, d)
    ws = workspace(nb, "local")
    nat.call("abc_local_fit", p(X), p(w), N, d, int(k), float(scaling),
             float(eps), p(covs), p(inv), p(dets), p(chol), p(lnorm), p(ws),
             ws.numel(), stream_ptr())
    return covs, inv, dets, chol, lnorm


def local_logpdf(x, X, w, inv, lnorm, out=None):
    M, d = x.shape
    N = X.shape[0]
    out = torch.empty(M, dtype=F64, device=x.device) if out is None else out
    if M == 0:
        return out
    ws = workspace(nat.query("abc_local_logpdf_workspace", M, N, d), "local_pdf")
    nat.call("abc_local_logpdf", p(x), M, p(X), p(w), N, d, p(inv), p(lnorm),
             p(out), p(ws), ws.numel(), stream_ptr())
    return out


LOG_2PI = math.log(2 * math.pi)


# ---- stochastic acceptance -------------------------------------------------

KERNEL_KINDS = {"independent_normal": 0, "independent_laplace": 1,
                "normal": 2, "poisson": 3, "binomial": 4,
                "negative_binomial": 5}


def kernel_logpdf(x, cols, x0k, kind, par, c, U=None, ret_lin=False,
                  out=None):
    """StochasticKernel values pdf(x_0 | x) for every row of x [B, S]
    (abc_kernel_logpdf); cols / x0k / par / U are device tensors in the
    kernel's key order."""
    B, S = x.shape
    K = int(cols.numel())
    r = 0 if U is None else int(U.shape[1])
    out = torch.empty(B, dtype=F64, device=x.device) if out is None else out
    nat.call("abc_kernel_logpdf", p(x), B, S, p(cols), K, p(x0k),
             KERNEL_KINDS[kind], p(par), p(U), r, float(c), int(bool(ret_lin)),
             p(out), stream_ptr())
    return out


def stochastic_accept(dens, pdf_norm, temperature, scale_log, apply_iw, seed,
                      generation, idx0):
    """(key, acceptance weight) per candidate (abc_stochastic_accept):
    accepted iff key <= 0."""
    B = dens.numel()
    key = torch.empty(B, dtype=F64, device=dens.device)
    accw = torch.empty(B, dtype=F64, device=dens.device)
    nat.call("abc_stochastic_accept", p(dens), B, float(pdf_norm),
             float(temperature), int(bool(scale_log)), int(bool(apply_iw)),
             int(seed) & (2 ** 64 - 1), int(generation) & 0xFFFFFFFF,
             int(idx0), p(key), p(accw), stream_ptr())
    return key, accw


TEMPER_ACCEPTANCE, TEMPER_ESS, TEMPER_MAX, TEMPER_ACCEPTANCE_LIN = 0, 1, 2, 3


def temper_sums(dens, lr, pdf_norm, scale_log, mode, beta=0.0, shift=0.0,
                lr_sub=None):
    """Two device reductions over R records (abc_temper_sums); returns the
    host pair (a, b), see include/abcgpu.h."""
    R = lr.numel()
    if lr_sub is not None and lr_sub.numel() != R:
        raise ValueError("temper_sums: lr / lr_sub sizes differ")
    out = torch.empty(2, dtype=F64, device=lr.device)
    ws = workspace(nat.query("abc_temper_workspace"), "temper")
    nat.call("abc_temper_sums", p(dens), p(lr), p(lr_sub), R, float(pdf_norm),
             int(bool(scale_log)), int(mode), float(beta), float(shift),
             p(out), p(ws), ws.numel(), stream_ptr())
    a, b = out.cpu().numpy()
    return float(a), float(b)
