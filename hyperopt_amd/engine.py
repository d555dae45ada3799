"""Host-side mirror of the reference's TPE operator interface, running on the
gfx950 HIP engine through the C ABI (include/hyperopt_tpe.h).

`GMM1_lpdf`, `LGMM1_lpdf`, `categorical_lpdf`, `broadcast_best`, `GMM1`,
`LGMM1` and `categorical` keep the argument meaning and the error behaviour of
the reference functions they replace (hyperopt/tpe.py:56-307, 769-778 and
hyperopt/pyll/stochastic.py:109-147); `Engine` holds a device context with a
resident posterior and runs fused suggestion rounds.
"""
import ctypes
import threading

import numpy as np

from . import _lib as L


class EngineError(RuntimeError):
    pass


def _raise(code, msg):
    msg = msg.decode() if isinstance(msg, bytes) else msg
    if code == L.TPE_ERR_VALUE:
        raise ValueError(msg)
    if code == L.TPE_ERR_TYPE:
        raise TypeError(msg)
    raise EngineError('%s (code %d)' % (msg, code))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


RESULT_DTYPE = np.dtype([('value', '<f8'), ('score', '<f8'), ('lpdf_below', '<f8'),
                         ('lpdf_above', '<f8'), ('index', '<i8'), ('label', '<i4'),
                         ('status', '<i4')])
assert RESULT_DTYPE.itemsize == ctypes.sizeof(L.LabelResult)

DESC_DTYPE = np.dtype([('kind', '<i4'), ('flags', '<i4'), ('low', '<f8'), ('high', '<f8'),
                       ('q', '<f8'), ('below_off', '<i8'), ('above_off', '<i8'),
                       ('n_below', '<i4'), ('n_above', '<i4')])
assert DESC_DTYPE.itemsize == ctypes.sizeof(L.LabelDesc)


SPEC_DTYPE = np.dtype([('kind', '<i4'), ('flags', '<i4'), ('low', '<f8'), ('high', '<f8'),
                       ('q', '<f8'), ('prior_mu', '<f8'), ('prior_sigma', '<f8'),
                       ('upper', '<i4'), ('randint', '<i4'), ('p_off', '<i8'),
                       ('stream', '<i4'), ('reserved', '<i4')])
assert SPEC_DTYPE.itemsize == ctypes.sizeof(L.LabelSpec)


def bounds_flags(low, high, q):
    f = 0
    if low is not None:
        f |= L.TPE_HAS_LOW
    if high is not None:
        f |= L.TPE_HAS_HIGH
    if q is not None:
        f |= L.TPE_HAS_Q
    return f


DEFAULT_LF = 25   # tpe.py:35: adaptive_parzen_normal's LF and ap_filter_trials' gamma_cap


def _check_lf(lf):
    """The builds cap n_below at gamma_cap = DEFAULT_LF (tpe.py:626, 636)
    and weight the Parzen components with linear forgetting `lf`
    (tpe.py:406): with lf >= DEFAULT_LF every below mixture keeps equal
    weights, the only case in which the reference (and so the tie order it
    fixes) is defined -- tpe.suggest never passes another."""
    if int(lf) < DEFAULT_LF:
        raise ValueError('linear forgetting %d < gamma_cap %d: a below mixture would depend on '
                         'the order of its observations' % (int(lf), DEFAULT_LF))


def _devices(device):
    if isinstance(device, (list, tuple)):
        if not device:
            raise ValueError('devices must not be empty')
        return tuple(int(d) for d in device)
    return (int(device),)


class Engine(object):
    """A device context: one GPU and HIP stream, or -- `device` a list of
    ordinals -- a multi-device context whose suggestion rounds are split over
    the GPUs with bit-identical results (tpe_ctx_create_multi).  Not
    thread-safe; the module-level helpers keep one Engine per (thread,
    devices, precision)."""

    def __init__(self, device=0, precision='f64'):
        self.lib = L.load()
        self.precision = precision
        prec = {'f64': L.TPE_F64, 'f32': L.TPE_F32}[precision]
        devs = _devices(device)
        h = ctypes.c_void_p()
        if len(devs) == 1:
            rc = self.lib.tpe_ctx_create(devs[0], prec, ctypes.byref(h))
        else:
            arr = (ctypes.c_int * len(devs))(*devs)
            rc = self.lib.tpe_ctx_create_multi(arr, len(devs), prec, ctypes.byref(h))
        if rc != L.TPE_OK:
            raise EngineError('tpe_ctx_create(devices=%s): %s' % (
                list(devs), self.lib.tpe_last_error(None).decode()))
        self.h = h
        self.devices = devs
        self.device = devs[0]
        self.n_labels = 0
        # bumped by every call that replaces the device-resident history, so
        # a DeviceHistoryUploader can tell its history is no longer there
        self.history_generation = 0

    def close(self):
        if getattr(self, 'h', None):
            self.lib.tpe_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != L.TPE_OK:
            _raise(rc, self.lib.tpe_last_error(self.h))

    # -- resident posterior --------------------------------------------------
    def set_posterior(self, descs, weights, mus, sigmas):
        """descs: structured array of DESC_DTYPE (one row per label)."""
        descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
        w, m, s = _f64(weights), _f64(mus), _f64(sigmas)
        self._check(self.lib.tpe_set_posterior(self.h, _ptr(descs), len(descs), _ptr(w),
                                               _ptr(m), _ptr(s), len(w)))
        self.n_labels = len(descs)

    def build_posterior(self, specs, cat_p, losses, obs_off, obs_trial, obs_val, gamma,
                        prior_weight, lf=25, tie_order='reference'):
        """Device posterior build from the history: specs is a SPEC_DTYPE
        array, observations in CSR form (obs_off per label; obs_trial =
        position in `losses`, -1 for none; obs_val already transformed).
        tie_order 'reference' (default): reset + append + the ordered build,
        with numpy's np.argsort order wherever a mixture depends on the order
        of ties (posterior.build_reference_order); 'position': one
        tpe_build_posterior call, ties by position.  Returns n_below."""
        from . import posterior as _post
        _check_lf(lf)
        specs = np.ascontiguousarray(specs, dtype=SPEC_DTYPE)
        cat_p = _f64(cat_p)
        losses = _f64(losses)
        obs_off = np.ascontiguousarray(obs_off, dtype=np.int64)
        obs_trial = np.ascontiguousarray(obs_trial, dtype=np.int32)
        obs_val = _f64(obs_val)
        if tie_order == 'reference':
            self.history_reset(specs, cat_p)
            self.history_append(np.diff(obs_off), obs_trial, obs_val)
            n_valid = int(np.count_nonzero(losses == losses))
            nb, self.tie_labels = _post.build_reference_order(
                self, losses, n_valid, gamma, prior_weight, lf, _post._ObsOf(obs_off, obs_trial, obs_val))
            return nb
        if tie_order != 'position':
            raise ValueError("tie_order must be 'reference' or 'position'")
        nb = ctypes.c_int32()
        self.history_generation += 1      # tpe_build_posterior resets the resident history
        self._check(self.lib.tpe_build_posterior(
            self.h, _ptr(specs), len(specs), _ptr(cat_p), len(cat_p), _ptr(losses), len(losses),
            _ptr(obs_off), _ptr(obs_trial), _ptr(obs_val), float(gamma), float(prior_weight),
            int(lf), ctypes.byref(nb)))
        self.n_labels = self.hist_labels = len(specs)
        return nb.value

    # -- device-resident history -----------------------------------------------
    def history_reset(self, specs, cat_p):
        specs = np.ascontiguousarray(specs, dtype=SPEC_DTYPE)
        cat_p = _f64(cat_p)
        self.history_generation += 1
        self._check(self.lib.tpe_history_reset(self.h, _ptr(specs), len(specs), _ptr(cat_p),
                                               len(cat_p)))
        self.hist_labels = len(specs)

    def history_append(self, n_new, obs_trial, obs_val):
        """n_new[l] new observations of label l (concatenated label-major):
        trial positions (tid order) and transformed values."""
        n_new = np.ascontiguousarray(n_new, dtype=np.int64)
        obs_trial = np.ascontiguousarray(obs_trial, dtype=np.int32)
        obs_val = _f64(obs_val)
        self._check(self.lib.tpe_history_append(self.h, _ptr(n_new), _ptr(obs_trial),
                                                _ptr(obs_val)))

    def build_posterior_resident(self, losses, n_valid, gamma, prior_weight, lf=25):
        """Rebuild the posterior from the resident history; losses per trial
        position, NaN for a trial outside the history.  Returns n_below."""
        _check_lf(lf)
        losses = _f64(losses)
        nb = ctypes.c_int32()
        self._check(self.lib.tpe_build_posterior_resident(
            self.h, _ptr(losses), len(losses), int(n_valid), float(gamma), float(prior_weight),
            int(lf), ctypes.byref(nb)))
        self.n_labels = self.hist_labels
        return nb.value

    def build_posterior_ordered(self, losses, n_valid, gamma, prior_weight, lf=25, below=None,
                                order_off=None, order=None):
        """build_posterior_resident with the reference's tie order where the
        caller supplies it (tpe_build_posterior_resident_ordered): `below` a
        uint8 mask per trial position, `order_off` / `order` per label the
        np.argsort of its above observations.  Returns (n_below, ties):
        ties[l] bit 1 (bit 0) when label l's above (below) mixture depends on
        a tie order that was not supplied, ties[-1] when equal losses
        straddle the split."""
        _check_lf(lf)
        losses = _f64(losses)
        L_ = self.hist_labels
        if below is not None:
            below = np.ascontiguousarray(below, dtype=np.uint8)
            if len(below) != len(losses):
                raise ValueError('below mask must cover every trial position')
        if order_off is not None:
            order_off = np.ascontiguousarray(order_off, dtype=np.int64)
            order = np.ascontiguousarray(order, dtype=np.int32)
            if len(order_off) != L_ + 1 or order_off[-1] != len(order):
                raise ValueError('order offsets must be n_labels + 1 long and end at len(order)')
        nb = ctypes.c_int32()
        ties = np.zeros(L_ + 1, dtype=np.int32)
        self._check(self.lib.tpe_build_posterior_resident_ordered(
            self.h, _ptr(losses), len(losses), int(n_valid), float(gamma), float(prior_weight),
            int(lf), _ptr(below), _ptr(order_off), _ptr(order), ctypes.byref(nb), _ptr(ties)))
        self.n_labels = self.hist_labels
        return nb.value, ties

    def rebuild_labels(self, losses, n_valid, gamma, prior_weight, lf, order_off, order, labels,
                       defer=False):
        """The ordered rebuild of `labels` only (tpe_rebuild_labels), right
        after a build of the same history and arguments; the other labels
        and the below set are kept.  Returns (n_below, ties).  defer: a
        rebuild of quantized / categorical labels only returns without
        waiting for its report (TPE_OPT_DEFER_REPORT; ties then zeros): the
        next round applies it after queuing the dense labels' kernels, and
        build_report() returns the real ties."""
        _check_lf(lf)
        losses = _f64(losses)
        L_ = self.hist_labels
        order_off = np.ascontiguousarray(order_off, dtype=np.int64)
        order = np.ascontiguousarray(order, dtype=np.int32)
        if len(order_off) != L_ + 1 or order_off[-1] != len(order):
            raise ValueError('order offsets must be n_labels + 1 long and end at len(order)')
        only = np.ascontiguousarray(sorted(int(l) for l in labels), dtype=np.int32)
        nb = ctypes.c_int32()
        ties = np.zeros(L_ + 1, dtype=np.int32)
        if defer:
            self.set_option('defer_report', 1)   # (consumed by this rebuild)
        self._check(self.lib.tpe_rebuild_labels(
            self.h, _ptr(losses), len(losses), int(n_valid), float(gamma), float(prior_weight), int(lf),
            _ptr(order_off), _ptr(order), _ptr(only), len(only), ctypes.byref(nb), _ptr(ties)))
        return nb.value, ties

    def build_report(self):
        """(n_below, ties) of the last build, applying a deferred rebuild's
        report first (tpe_build_report)."""
        nb = ctypes.c_int32()
        ties = np.zeros(self.hist_labels + 1, dtype=np.int32)
        self._check(self.lib.tpe_build_report(self.h, ctypes.byref(nb), _ptr(ties)))
        return nb.value, ties

    def get_mixture(self, label, side):
        """(weights, mus, sigmas) of a built mixture (side 0 below, 1 above)."""
        n = ctypes.c_int32()
        self._check(self.lib.tpe_get_mixture(self.h, int(label), int(side), None, None, None, 0,
                                             ctypes.byref(n)))
        w, m, s = np.empty(n.value), np.empty(n.value), np.empty(n.value)
        self._check(self.lib.tpe_get_mixture(self.h, int(label), int(side), _ptr(w), _ptr(m),
                                             _ptr(s), n.value, ctypes.byref(n)))
        return w, m, s

    def prepare(self, n_candidates, n_rounds=1):
        """Build the expansion index of the resident posterior now
        (tpe_prepare; the first round(s) of n_candidates would build it)."""
        self._check(self.lib.tpe_prepare(self.h, int(n_candidates), int(n_rounds)))

    def arm_prepare(self, n_candidates, n_rounds=1):
        """Have the next device build of the resident history queue the
        expansion index itself, before it returns (tpe_arm_prepare)."""
        self._check(self.lib.tpe_arm_prepare(self.h, int(n_candidates), int(n_rounds)))

    def last_build_ms(self):
        ms = ctypes.c_float()
        self._check(self.lib.tpe_last_build_ms(self.h, ctypes.byref(ms)))
        return ms.value

    def _labels(self):
        """Rows tpe_suggest writes per round: asked from the library, so an
        output buffer can never be shorter than the resident posterior."""
        self.n_labels = int(self.lib.tpe_resident_labels(self.h))
        return self.n_labels

    def suggest(self, seed, n_candidates, round=0, cand_offset=0):
        out = np.empty(self._labels(), dtype=RESULT_DTYPE)   # (every record written)
        self._check(self.lib.tpe_suggest(self.h, int(seed) & 0xFFFFFFFFFFFFFFFF,
                                         int(round) & 0xFFFFFFFF, int(n_candidates),
                                         int(cand_offset), _ptr(out)))
        return out

    def suggest_batch(self, seed, rounds, n_candidates, cand_offset=0):
        rounds = np.ascontiguousarray(np.asarray(rounds, dtype=np.uint32))
        # (every record written: np.zeros cost 0.17-1.6 ms at config 5's 25 MB)
        out = np.empty(len(rounds) * self._labels(), dtype=RESULT_DTYPE)
        self._check(self.lib.tpe_suggest_batch(self.h, int(seed) & 0xFFFFFFFFFFFFFFFF,
                                               _ptr(rounds), len(rounds), int(n_candidates),
                                               int(cand_offset), _ptr(out)))
        return out.reshape(len(rounds), self.n_labels)

    def suggest_batch_device(self, seed, rounds, n_candidates, d_out, cand_offset=0):
        """tpe_suggest_batch into a device buffer: d_out a torch uint8 tensor
        on this engine's GPU holding len(rounds) * n_labels records
        (RESULT_DTYPE bytes), complete on return -- for an RCCL all-gather
        without a host round trip."""
        rounds = np.ascontiguousarray(np.asarray(rounds, dtype=np.uint32))
        need = len(rounds) * self._labels() * RESULT_DTYPE.itemsize
        if not d_out.is_cuda or d_out.numel() * d_out.element_size() < need or not d_out.is_contiguous():
            raise ValueError('d_out must be a contiguous device tensor of %d bytes' % need)
        self._check_device(d_out, 'd_out')
        _torch_stream_done(d_out)
        self._check(self.lib.tpe_suggest_batch_device(
            self.h, int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(rounds), len(rounds), int(n_candidates),
            int(cand_offset), ctypes.c_void_p(d_out.data_ptr()), None))
        return d_out

    def _check_device(self, t, what):
        """The device entry points copy on this context's stream: a buffer
        on another GPU would be written across devices (or fault)."""
        if len(self.devices) != 1 or t.device.index != self.device:
            raise ValueError('%s is on cuda:%s, this engine runs on cuda:%d%s'
                             % (what, t.device.index, self.device,
                                '' if len(self.devices) == 1 else ' (multi-device contexts take host buffers)'))

    def merge_results_device(self, d_parts, n_parts, n, d_out):
        """tpe_merge_results over device tensors (n_parts blocks of n records
        -> n records), on this engine's GPU."""
        rec = RESULT_DTYPE.itemsize
        for t, need, what in ((d_parts, n_parts * n * rec, 'd_parts'), (d_out, n * rec, 'd_out')):
            if not t.is_cuda or t.numel() * t.element_size() < need or not t.is_contiguous():
                raise ValueError('%s must be a contiguous device tensor of %d bytes' % (what, need))
            self._check_device(t, what)
        _torch_stream_done(d_parts)
        self._check(self.lib.tpe_merge_results_device(
            self.h, ctypes.c_void_p(d_parts.data_ptr()), int(n_parts), int(n),
            ctypes.c_void_p(d_out.data_ptr())))
        return d_out

    def export_size(self):
        """Bytes tpe_export_posterior writes for the resident posterior (its
        expansion index queued first when the rounds would use one)."""
        n = ctypes.c_int64()
        self._check(self.lib.tpe_export_posterior(self.h, None, 0, ctypes.byref(n)))
        return int(n.value)

    def export_posterior(self, d_out):
        """The resident posterior and its expansion index as one blob in
        d_out (a contiguous device uint8 tensor on this engine's GPU, at
        least export_size() bytes), complete on return; returns its size."""
        n = ctypes.c_int64()
        cap = d_out.numel() * d_out.element_size()
        if not d_out.is_cuda or not d_out.is_contiguous():
            raise ValueError('d_out must be a contiguous device tensor')
        self._check_device(d_out, 'd_out')
        _torch_stream_done(d_out)
        self._check(self.lib.tpe_export_posterior(self.h, ctypes.c_void_p(d_out.data_ptr()), cap,
                                                  ctypes.byref(n)))
        if n.value > cap:
            raise ValueError('d_out holds %d bytes, the posterior needs %d' % (cap, n.value))
        return int(n.value)

    def import_posterior(self, d_blobs, part_off, part_labels):
        """Resident posterior = the labels of the blobs in d_blobs (device
        uint8 tensor on this engine's GPU): part p at byte part_off[p] holds
        the labels part_labels[p] (their space indices, in the exporter's
        label order); together the label lists cover 0..L-1 once."""
        if not d_blobs.is_cuda or not d_blobs.is_contiguous():
            raise ValueError('d_blobs must be a contiguous device tensor')
        self._check_device(d_blobs, 'd_blobs')
        off = np.ascontiguousarray(np.asarray(part_off, dtype=np.int64))
        counts = np.ascontiguousarray(np.asarray([len(p) for p in part_labels], dtype=np.int32))
        ids = np.ascontiguousarray(np.concatenate([np.asarray(p, dtype=np.int32) for p in part_labels]))
        if len(off) != len(counts):
            raise ValueError('one offset per part')
        _torch_stream_done(d_blobs)
        self._check(self.lib.tpe_import_posterior(
            self.h, ctypes.c_void_p(d_blobs.data_ptr()), d_blobs.numel() * d_blobs.element_size(),
            _ptr(off), len(off), _ptr(counts), _ptr(ids)))
        self._labels()

    def score(self, label, cand, want_lpdf=True):
        cand = _f64(cand).ravel()
        lb = np.empty(len(cand)) if want_lpdf else None
        la = np.empty(len(cand)) if want_lpdf else None
        out = np.zeros(1, dtype=RESULT_DTYPE)
        self._check(self.lib.tpe_score(self.h, int(label), _ptr(cand), len(cand), _ptr(lb),
                                       _ptr(la), _ptr(out)))
        return lb, la, out[0]

    def last_timing(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        self._check(self.lib.tpe_last_timing(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def last_evals(self):
        return int(self.lib.tpe_last_evals(self.h))

    def last_screen(self, with_ms=False):
        """(candidates screened in fp32, candidates re-scored in fp64) of the
        last round ((0, 0) when the round was not screened); with_ms adds the
        device ms of the fp32 screening kernel."""
        a, b, ms = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_float()
        self._check(self.lib.tpe_last_screen(self.h, ctypes.byref(a), ctypes.byref(b),
                                             ctypes.byref(ms)))
        return (a.value, b.value, ms.value) if with_ms else (a.value, b.value)

    def last_screen_terms(self):
        """(candidate, component) terms the last round's screen summed over
        both mixtures (the windowed screen skips the components that cannot
        matter to a tile)."""
        t = ctypes.c_int64()
        self._check(self.lib.tpe_last_screen_terms(self.h, ctypes.byref(t)))
        return t.value

    def last_screen_mode(self):
        """0 none, 1 plain fp32 screen, 2 windowed fp32 screen, 3 expansion
        screen (the last round's dense tile-map labels)."""
        return int(self.lib.tpe_last_screen_mode(self.h))

    def last_hot(self):
        """(candidates the hot-bin prefilter listed for the expansion screen,
        fallback) of the last round; listed is -1 when the prefilter did not
        run, fallback 1 when the round screened every candidate instead."""
        a, b = ctypes.c_int64(), ctypes.c_int32()
        self._check(self.lib.tpe_last_hot(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def last_prepare_ms(self):
        """Wall ms of the last build of the expansion screen's index (once per
        posterior, before its first large sampled round)."""
        ms = ctypes.c_float()
        self._check(self.lib.tpe_last_prepare(self.h, ctypes.byref(ms)))
        return ms.value

    def device_bytes(self):
        """Device memory the library holds (every context of the process),
        bytes: the high-water mark of its buffers (tpe_device_bytes)."""
        return int(self.lib.tpe_device_bytes())

    def last_drawn(self):
        """(quantized, categorical) candidates the last round drew: fewer
        than rounds x n when the exact early exit stopped a label's round."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.tpe_last_drawn(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def last_rescore_terms(self):
        """(candidate, component) terms the last round's fp64 re-score
        evaluated (every re-scored candidate over both of its mixtures)."""
        t = ctypes.c_int64()
        self._check(self.lib.tpe_last_rescore_terms(self.h, ctypes.byref(t)))
        return t.value

    OPTIONS = {'screen': L.TPE_OPT_SCREEN, 'splitk': L.TPE_OPT_SPLITK, 'dedup': L.TPE_OPT_DEDUP,
               'chunks': L.TPE_OPT_CHUNKS, 'whole_n': L.TPE_OPT_WHOLE_N,
               'whole_rounds': L.TPE_OPT_WHOLE_ROUNDS, 'timing': L.TPE_OPT_TIMING,
               'window': L.TPE_OPT_WINDOW, 'win_t': L.TPE_OPT_WIN_T,
               'win_groups': L.TPE_OPT_WIN_GROUPS, 'expand': L.TPE_OPT_EXPAND,
               'hot': L.TPE_OPT_HOT, 'early': L.TPE_OPT_EARLY, 'hot_div': L.TPE_OPT_HOT_DIV,
               'zero_win': L.TPE_OPT_ZERO_WIN, 'value_only': L.TPE_OPT_VALUE_ONLY,
               'rescore_cap': L.TPE_OPT_RESCORE_CAP, 'mode_mask': L.TPE_OPT_MODE_MASK,
               'aux_families': L.TPE_OPT_AUX_FAMILIES,
               'bx_split': L.TPE_OPT_BX_SPLIT, 'bx_t': L.TPE_OPT_BX_T,
               'pk_sliced': L.TPE_OPT_PK_SLICED, 'defer_report': L.TPE_OPT_DEFER_REPORT,
               'label_shards': L.TPE_OPT_LABEL_SHARDS}

    def set_option(self, name, value):
        """Engine switches (include/hyperopt_tpe.h TPE_OPT_*): 'screen',
        'splitk', 'dedup', 'timing', 'window', 'expand', 'hot', 'early',
        'value_only' (bool: batched rounds report the winner's index and value
        only where the screen alone decided it, lpdfs NaN), 'chunks'
        (int, 0 = auto), 'hot_div' (the prefilter's list length n / hot_div),
        'win_t' (the windowed screen's cut, 8..62), 'win_groups' (label
        groups pipelined over two streams, 0 = auto),
        'whole_n' / 'whole_rounds' (the whole problem when this engine runs
        one shard of it, 0 = the call's own)."""
        self._check(self.lib.tpe_set_option(self.h, self.OPTIONS[name], int(value)))

    def screen_probe(self, label, cand):
        """fp32 screen score and its error bound for supplied candidates of a
        dense resident label (diagnostic, tpe_screen_probe)."""
        cand = _f64(cand).ravel()
        s, e = np.empty(len(cand)), np.empty(len(cand))
        self._check(self.lib.tpe_screen_probe(self.h, int(label), _ptr(cand), len(cand), _ptr(s),
                                              _ptr(e)))
        return s, e

    def hot_probe(self, label, cand):
        """(upper, lower, mass): the fp64 score's interval over each supplied
        candidate's sub-bin and the sub-bin's sampling mass (the hot-bin
        prefilter's table, tpe_hot_probe)."""
        cand = _f64(cand).ravel()
        u, l, m = np.empty(len(cand)), np.empty(len(cand)), np.empty(len(cand))
        self._check(self.lib.tpe_hot_probe(self.h, int(label), _ptr(cand), len(cand), _ptr(u), _ptr(l),
                                           _ptr(m)))
        return u, l, m

    # slot 0: dense GMM1 -- and, in sampled tile/packed rounds, the dense
    # LGMM1 labels too (one merged launch; slot 1 then stays 0)
    MODES = ('dense', 'dense_lgmm1', 'quant_gmm1', 'quant_lgmm1', 'categorical')

    def last_mode_stats(self):
        """{family: (device_ms, evals)} of the last round."""
        ms = np.zeros(5, dtype=np.float32)
        ev = np.zeros(5, dtype=np.int64)
        self._check(self.lib.tpe_last_mode_stats(self.h, _ptr(ms), _ptr(ev)))
        return {m: (float(ms[i]), int(ev[i])) for i, m in enumerate(self.MODES)}

    # -- single reference ops --------------------------------------------------
    def _mix_lpdf(self, fn, samples, weights, mus, sigmas, low, high, q):
        samples = np.asarray(samples, dtype=np.float64)
        weights, mus, sigmas = (np.asarray(a, dtype=np.float64) for a in (weights, mus, sigmas))
        if samples.size == 0:
            return np.asarray([])
        for nm, a in (('weights', weights), ('mus', mus), ('sigmas', sigmas)):
            if a.ndim != 1:
                raise TypeError('need vector of %s' % nm, a.shape)
        assert len(weights) == len(mus) == len(sigmas)
        x = np.ascontiguousarray(samples.ravel())
        out = np.empty(x.shape)
        self._check(fn(self.h, _ptr(x), len(x), _ptr(_f64(weights)), _ptr(_f64(mus)),
                       _ptr(_f64(sigmas)), len(weights), bounds_flags(low, high, q),
                       float(low or 0.0), float(high or 0.0), float(q or 0.0), _ptr(out)))
        return out.reshape(samples.shape)

    def GMM1_lpdf(self, samples, weights, mus, sigmas, low=None, high=None, q=None):
        return self._mix_lpdf(self.lib.tpe_gmm1_lpdf, samples, weights, mus, sigmas, low, high, q)

    def LGMM1_lpdf(self, samples, weights, mus, sigmas, low=None, high=None, q=None):
        return self._mix_lpdf(self.lib.tpe_lgmm1_lpdf, samples, weights, mus, sigmas, low, high, q)

    def categorical_lpdf(self, sample, p, upper=None):
        sample = np.asarray(sample)
        if sample.size == 0:
            return np.asarray([])
        p = _f64(p)
        s = np.ascontiguousarray(sample.ravel().astype(np.int64))
        out = np.empty(s.shape)
        self._check(self.lib.tpe_categorical_lpdf(self.h, _ptr(s), len(s), _ptr(p), len(p),
                                                  _ptr(out)))
        return out.reshape(sample.shape)

    def broadcast_best(self, samples, below_llik, above_llik):
        if len(samples):
            b, a = _f64(below_llik).ravel(), _f64(above_llik).ravel()
            if len(samples) != len(b) or len(b) != len(a):
                raise ValueError()
            best = ctypes.c_int64()
            self._check(self.lib.tpe_broadcast_best(self.h, _ptr(b), _ptr(a), len(b),
                                                    ctypes.byref(best)))
            return [samples[best.value]] * len(samples)
        return []

    def _mix_sample(self, fn, weights, mus, sigmas, low, high, q, seed, size, stream, round,
                    offset):
        weights, mus, sigmas = (_f64(a) for a in (weights, mus, sigmas))
        assert len(weights) == len(mus) == len(sigmas)
        n = int(np.prod(size))
        out = np.empty(n)
        self._check(fn(self.h, _ptr(weights), _ptr(mus), _ptr(sigmas), len(weights),
                       bounds_flags(low, high, q), float(low or 0.0), float(high or 0.0),
                       float(q or 0.0), int(seed), int(stream), int(round), int(offset), n,
                       _ptr(out)))
        return out.reshape(size)

    def GMM1(self, weights, mus, sigmas, low=None, high=None, q=None, seed=0, size=(),
             stream=0, round=0, offset=0):
        return self._mix_sample(self.lib.tpe_gmm1_sample, weights, mus, sigmas, low, high, q,
                                seed, size, stream, round, offset)

    def LGMM1(self, weights, mus, sigmas, low=None, high=None, q=None, seed=0, size=(),
              stream=0, round=0, offset=0):
        return self._mix_sample(self.lib.tpe_lgmm1_sample, weights, mus, sigmas, low, high, q,
                                seed, size, stream, round, offset)

    def categorical(self, p, upper=None, seed=0, size=(), stream=0, round=0, offset=0):
        p = _f64(p)
        n = int(np.prod(size)) if size != () else 1
        out = np.empty(n, dtype=np.int64)
        self._check(self.lib.tpe_categorical_sample(self.h, _ptr(p), len(p), int(seed),
                                                    int(stream), int(round), int(offset), n,
                                                    _ptr(out)))
        return out.reshape(size if size != () else (1,))


def _torch_stream_done(t):
    """The device entry points run on the context's own stream: work torch
    queued on its current stream for these buffers (the H2D copy that filled
    them, the RCCL all-gather that wrote them, a read of the previous round)
    must be complete before the call.  (Round 4's first GPU run merged a
    buffer whose H2D copy had not landed.)"""
    import torch
    torch.cuda.current_stream(t.device).synchronize()


def merge_results(parts):
    """Merge per-shard winners (n_parts x n) with the broadcast_best order."""
    lib = L.load()
    parts = np.ascontiguousarray(parts, dtype=RESULT_DTYPE)
    if parts.ndim == 1:
        parts = parts[None]
    out = np.zeros(parts.shape[1], dtype=RESULT_DTYPE)
    rc = lib.tpe_merge_results(_ptr(parts), parts.shape[0], parts.shape[1], _ptr(out))
    if rc != L.TPE_OK:
        raise EngineError('tpe_merge_results failed (%d)' % rc)
    return out


_tls = threading.local()


def get_engine(device=0, precision='f64', role='main'):
    """Per-thread cached Engine (contexts are not thread-safe); `device` an
    ordinal or a list of them; `role` keeps separate contexts -- hence
    separate device-resident histories -- for callers that would otherwise
    evict each other's (tpe.suggest's batch='pending' views)."""
    cache = getattr(_tls, 'engines', None)
    if cache is None:
        cache = _tls.engines = {}
    key = (_devices(device), precision, role)
    if key not in cache:
        eng = Engine(device, precision)
        eng.set_option('timing', 0)          # tpe.suggest reads no device timings
        if len(_devices(device)) == 1:
            # tpe.suggest reads the winners' values only (tpe.py:906-916):
            # no lpdfs for a batched round the screen alone decided (a
            # multi-device context merges its shards by score: exact there)
            eng.set_option('value_only', 1)
            # the quantized and categorical labels beside the dense draw on
            # the second stream (same documents; only their draw-count
            # statistics depend on the interleaving, and tpe.suggest reads none)
            eng.set_option('aux_families', 1)
        cache[key] = eng
    return cache[key]
