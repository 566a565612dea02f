"""Python face of the native engine: numpy in, numpy out, over the C ABI.

One ``Engine`` = one HIP device's share of a model: the user rows it owns,
every item row, the Adagrad accumulators, the HBM-resident interaction graph
and the device sampler position.  The model classes (bprmf.py, gbprmf.py,
cml.py, amf.py) and the samplers are thin wrappers over this class.
"""
import ctypes

import numpy as np

from . import _native as N


def _ptr(a, ctype):
    return a.ctypes.data_as(ctypes.POINTER(ctype))


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _is_dev(x):
    """A torch tensor in HIP device memory (the C ABI takes its pointer as is)."""
    return hasattr(x, "data_ptr") and bool(getattr(x, "is_cuda", False))


def _dev(t, dtype, ctype):
    """Contiguous device tensor of ``dtype`` and its pointer; torch's stream is
    synchronised first, because the engine reads it on its own stream."""
    import torch
    t = t.to(dtype).contiguous()
    torch.cuda.current_stream(t.device).synchronize()
    return t, ctypes.cast(t.data_ptr(), ctypes.POINTER(ctype))


class _DevArg(object):
    """A device tensor plus its ctypes pointer (keeps the tensor alive)."""

    def __init__(self, t, p):
        self.t, self.p = t, p


def _arg(x, ctype):
    return x.p if isinstance(x, _DevArg) else _ptr(x, ctype)


class Engine(object):
    def __init__(self, model, n_users, n_items, n_factors, n_neg=1, gsize=1, lr=0.1,
                 reg=0.02, rho=0.5, margin=1.5, reg_cov=1.0, clip_norm=1.0, reg_adv=1.0,
                 epsilon=0.5, acc_init=0.1, use_rank_weight=True, device=0,
                 dense_item_apply=False, seed=20261015, plr_kind=None, alpha=1.0, beta=1.0,
                 gamma=1.0, amf_mode="reference"):
        L = N.lib()
        if isinstance(model, str):
            name = model.lower()
            model = N.MODEL_IDS[name]
            if name in ("prigp", "cplr"):   # tuple models: the tuple width fixes n_neg
                plr_kind = N.CF_PLR_PRIGP if name == "prigp" else N.CF_PLR_CPLR
        if int(model) == N.CF_PLR:
            plr_kind = N.CF_PLR_PRIGP if plr_kind is None else int(plr_kind)
            n_neg = 3 if plr_kind == N.CF_PLR_PRIGP else 2
        cfg = N.CfConfig()
        L.cf_config_defaults(ctypes.byref(cfg))
        cfg.model = int(model)
        cfg.n_factors = int(n_factors)
        cfg.n_users = int(n_users)
        cfg.n_items = int(n_items)
        cfg.n_neg = int(n_neg)
        cfg.gsize = int(gsize)
        cfg.lr = float(lr)
        cfg.reg = float(reg)
        cfg.rho = float(rho)
        cfg.margin = float(margin)
        cfg.reg_cov = float(reg_cov)
        cfg.clip_norm = float(clip_norm)
        cfg.reg_adv = float(reg_adv)
        cfg.epsilon = float(epsilon)
        cfg.acc_init = float(acc_init)
        cfg.use_rank_weight = 1 if use_rank_weight else 0
        cfg.device = int(device)
        cfg.dense_item_apply = 1 if dense_item_apply else 0
        cfg.plr_kind = int(plr_kind or 0)
        cfg.alpha, cfg.beta, cfg.gamma = float(alpha), float(beta), float(gamma)
        # AMF: "reference" (Δ = 0, what amf.py computes) or "apr" (Δ from the
        # normalised embedding-loss gradient, include/cf_engine.h amf_mode)
        cfg.amf_mode = N.AMF_MODES[amf_mode] if isinstance(amf_mode, str) else int(amf_mode)
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.cfg = cfg
        self.model = int(model)
        self.n_users, self.n_items, self.d = int(n_users), int(n_items), int(n_factors)
        self.n_neg = int(n_neg)
        self.gsize = int(gsize) if self.model == N.CF_GBPR else 0
        self.plr_kind = int(plr_kind or 0)
        self._h = ctypes.c_void_p()
        N.check(L.cf_create(ctypes.byref(cfg), ctypes.byref(self._h)), "cf_create")
        self._L = L
        self.nnz = 0

    # ---- lifecycle --------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._L.cf_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        N.check(self._L.cf_synchronize(self._h), "cf_synchronize")

    def set_stream(self, hip_stream_ptr):
        N.check(self._L.cf_set_stream(self._h, ctypes.c_void_p(hip_stream_ptr or None)),
                "cf_set_stream")

    # ---- data -----------------------------------------------------------------
    def set_interactions(self, indptr, indices):
        indptr = np.ascontiguousarray(indptr, dtype=np.int64)
        indices = _i32(indices)
        N.check(self._L.cf_set_interactions(self._h, _ptr(indptr, ctypes.c_int64),
                                            _ptr(indices, ctypes.c_int32), int(indices.shape[0])),
                "cf_set_interactions")
        self.nnz = int(indices.shape[0])

    def init_params(self, mean=0.0, stddev=0.1, truncated=True, seed=1):
        N.check(self._L.cf_init_params(self._h, float(mean), float(stddev), 1 if truncated else 0,
                                       int(seed) & 0xFFFFFFFFFFFFFFFF), "cf_init_params")

    def _table_shape(self, name):
        if name in ("user", "acc_user"):
            return (self.n_users, self.d)
        if name in ("item", "acc_item"):
            return (self.n_items, self.d)
        return (self.n_items,)

    def set_table(self, name, arr):
        a = np.ascontiguousarray(arr, dtype=np.float32)
        if a.shape != self._table_shape(name):
            raise ValueError("table %s must have shape %s" % (name, self._table_shape(name)))
        N.check(self._L.cf_set_table(self._h, N.TABLES[name], _ptr(a, ctypes.c_float), a.size),
                "cf_set_table(%s)" % name)

    def get_table(self, name):
        guard = getattr(self, "_stale_guard", None)
        if guard is not None and guard.stale and name in guard.stale_tables:
            # rs_ag item-range ownership: only the owner keeps its accumulator
            # rows current; the other ranks' copies are gathered by sync_state
            raise RuntimeError("%s is stale on this rank under the rs_ag item exchange: "
                               "call step.sync_state() before reading it" % name)
        out = np.empty(self._table_shape(name), dtype=np.float32)
        N.check(self._L.cf_get_table(self._h, N.TABLES[name], _ptr(out, ctypes.c_float), out.size),
                "cf_get_table(%s)" % name)
        return out

    PARAM_TABLES = ("user", "item", "bias", "acc_user", "acc_item", "acc_bias")

    def set_params(self, **tables):
        """cf_set_params: any of user, item, bias, acc_user, acc_item,
        acc_bias in one call (the others kept)."""
        bad = set(tables) - set(self.PARAM_TABLES)
        if bad:
            raise ValueError("unknown tables %s" % sorted(bad))
        keep, ptrs = [], []
        for name in self.PARAM_TABLES:
            a = tables.get(name)
            if a is None:
                ptrs.append(None)
                continue
            a = np.ascontiguousarray(a, dtype=np.float32)
            if a.shape != self._table_shape(name):
                raise ValueError("table %s must have shape %s" % (name, self._table_shape(name)))
            keep.append(a)
            ptrs.append(_ptr(a, ctypes.c_float))
        N.check(self._L.cf_set_params(self._h, *ptrs), "cf_set_params")

    def get_params(self, names=None):
        """cf_get_params: {name: array} for ``names`` (default every table
        the model has)."""
        has_bias = self.model in (N.CF_GBPR, N.CF_PLR)
        names = names or [t for t in self.PARAM_TABLES if has_bias or "bias" not in t]
        out = {n: np.empty(self._table_shape(n), dtype=np.float32) for n in names}
        N.check(self._L.cf_get_params(self._h, *[_ptr(out[t], ctypes.c_float) if t in out else None
                                                 for t in self.PARAM_TABLES]), "cf_get_params")
        return out

    # ---- training -------------------------------------------------------------
    def _batch(self, pairs, negs, groups):
        if _is_dev(pairs):   # torch device tensors: staged on the device (cf_step docs)
            import torch
            pairs, pp = _dev(pairs.reshape(-1, 2), torch.int32, ctypes.c_int32)
            B = pairs.shape[0]
            negs, npt = _dev(negs.reshape(B, -1), torch.int32, ctypes.c_int32)
            if negs.shape[1] != self.n_neg:
                raise ValueError("negs must have %d columns" % self.n_neg)
            gp = None
            if self.model == N.CF_GBPR:
                groups, gp = _dev(groups.reshape(B, -1), torch.int32, ctypes.c_int32)
                if groups.shape[1] != self.gsize:
                    raise ValueError("groups must have %d columns" % self.gsize)
            return B, _DevArg(pairs, pp), _DevArg(negs, npt), gp, groups
        pairs = _i32(pairs).reshape(-1, 2)
        B = pairs.shape[0]
        negs = _i32(negs).reshape(B, -1)
        if negs.shape[1] != self.n_neg:
            raise ValueError("negs must have %d columns" % self.n_neg)
        gp = None
        if self.model == N.CF_GBPR:
            groups = _i32(groups).reshape(B, -1)
            if groups.shape[1] != self.gsize:
                raise ValueError("groups must have %d columns" % self.gsize)
            gp = _ptr(groups, ctypes.c_int32)
        return B, pairs, negs, gp, groups

    def step(self, pairs, negs, groups=None, return_loss=True):
        B, pairs, negs, gp, _keep = self._batch(pairs, negs, groups)
        loss = ctypes.c_double(0.0)
        N.check(self._L.cf_step(self._h, _arg(pairs, ctypes.c_int32), _arg(negs, ctypes.c_int32),
                                gp, B, ctypes.byref(loss) if return_loss else None), "cf_step")
        return float(loss.value) if return_loss else None

    def step_plr(self, tuples, coefs=None, return_loss=True):
        """One host-fed tuple step (CF_PLR): tuples [B, n_neg + 2] int
        ((u,i,j,t,k) PRIGP / (u,i,t,j) CPLR), coefs [B, 2] float (CPLR);
        numpy arrays or torch device tensors."""
        if _is_dev(tuples):
            import torch
            t, tp = _dev(tuples, torch.int32, ctypes.c_int32)
            B, width = t.shape
            cp = None
            if coefs is not None:
                c, cp = _dev(coefs.reshape(B, 2), torch.float32, ctypes.c_float)
            out = ctypes.c_double(0.0)
            N.check(self._L.cf_step_plr(self._h, tp, int(width), cp, int(B),
                                        ctypes.byref(out) if return_loss else None), "cf_step_plr")
            return float(out.value) if return_loss else None
        t = _i32(tuples)
        B, width = t.shape
        cp = None
        if coefs is not None:
            c = np.ascontiguousarray(coefs, dtype=np.float32).reshape(B, 2)
            cp = _ptr(c, ctypes.c_float)
        out = ctypes.c_double(0.0)
        N.check(self._L.cf_step_plr(self._h, _ptr(t, ctypes.c_int32), int(width), cp, int(B),
                                    ctypes.byref(out) if return_loss else None), "cf_step_plr")
        return float(out.value) if return_loss else None

    def train_steps(self, batch_size, n_steps, return_loss=True):
        loss = ctypes.c_double(0.0)
        N.check(self._L.cf_train_steps(self._h, int(batch_size), int(n_steps),
                                       ctypes.byref(loss) if return_loss else None),
                "cf_train_steps")
        return float(loss.value) if return_loss else None

    def train_epoch(self, batch_size, return_loss=True):
        """One iteration of the reference's train loop (cf_train_epoch): the
        sampler's epoch to its end, returning the mean batch loss (TraLoss)."""
        loss = ctypes.c_double(0.0)
        N.check(self._L.cf_train_epoch(self._h, int(batch_size), ctypes.byref(loss) if return_loss else None),
                "cf_train_epoch")
        return float(loss.value) if return_loss else None

    def sample(self, batch_size):
        B = int(batch_size)
        pairs = np.empty((B, 2), dtype=np.int32)
        negs = np.empty((B, self.n_neg), dtype=np.int32)
        groups = np.empty((B, max(self.gsize, 1)), dtype=np.int32)
        N.check(self._L.cf_sample(self._h, B, _ptr(pairs, ctypes.c_int32),
                                  _ptr(negs, ctypes.c_int32),
                                  _ptr(groups, ctypes.c_int32) if self.gsize else None),
                "cf_sample")
        return pairs, negs, (groups if self.gsize else None)

    def sampler_state(self):
        e, b = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(self._L.cf_get_sampler_state(self._h, ctypes.byref(e), ctypes.byref(b)),
                "cf_get_sampler_state")
        return int(e.value), int(b.value)

    def set_sampler_state(self, epoch, batch):
        N.check(self._L.cf_set_sampler_state(self._h, int(epoch), int(batch)),
                "cf_set_sampler_state")

    def begin_phase(self, phase):
        N.check(self._L.cf_begin_phase(self._h, int(phase)), "cf_begin_phase")
        self._phase = int(phase)

    def apr_active(self):
        """AMF apr in its adversarial phase: a multi-rank step needs
        step_local_apr_embed + the all-reduce of the apr buffer first."""
        return self.cfg.amf_mode == N.CF_AMF_APR and getattr(self, "_phase", 0) == 1

    # ---- multi-rank split step -------------------------------------------------
    def bind_item_grad(self, device_ptr, n_elems):
        N.check(self._L.cf_bind_item_grad(self._h, ctypes.c_void_p(device_ptr), int(n_elems)),
                "cf_bind_item_grad")

    def step_local(self, batch_size=None, pairs=None, negs=None, groups=None):
        if pairs is None:
            N.check(self._L.cf_step_local(self._h, int(batch_size), None, None, None),
                    "cf_step_local")
            return
        B, pairs, negs, gp, _keep = self._batch(pairs, negs, groups)
        N.check(self._L.cf_step_local(self._h, B, _arg(pairs, ctypes.c_int32),
                                      _arg(negs, ctypes.c_int32), gp), "cf_step_local")

    def step_local_grad(self, batch_size=None, pairs=None, negs=None, groups=None):
        if pairs is None:
            N.check(self._L.cf_step_local_grad(self._h, int(batch_size), None, None, None),
                    "cf_step_local_grad")
            return
        B, pairs, negs, gp, _keep = self._batch(pairs, negs, groups)
        N.check(self._L.cf_step_local_grad(self._h, B, _arg(pairs, ctypes.c_int32),
                                           _arg(negs, ctypes.c_int32), gp), "cf_step_local_grad")

    def bind_apr_item_grad(self, device_ptr, n_elems):
        """The n_items * d buffer an apr step's item sums are all-reduced in
        (include/cf_engine.h cf_bind_apr_item_grad)."""
        N.check(self._L.cf_bind_apr_item_grad(self._h, ctypes.c_void_p(device_ptr), int(n_elems)),
                "cf_bind_apr_item_grad")

    def step_local_apr_embed(self, batch_size=None, pairs=None, negs=None):
        if pairs is None:
            N.check(self._L.cf_step_local_apr_embed(self._h, int(batch_size), None, None),
                    "cf_step_local_apr_embed")
            return int(batch_size)
        B, pairs, negs, _gp, _keep = self._batch(pairs, negs, None)
        N.check(self._L.cf_step_local_apr_embed(self._h, B, _arg(pairs, ctypes.c_int32),
                                                _arg(negs, ctypes.c_int32)), "cf_step_local_apr_embed")
        return B

    def step_local_apply(self, next_batch_size=0):
        N.check(self._L.cf_step_local_apply(self._h, int(next_batch_size)), "cf_step_local_apply")

    def step_item_reduce(self, piece):
        """Piece `piece` of the local step's item reduce (cf_set_option
        "item_pieces" > 1; include/cf_engine.h cf_step_item_reduce)."""
        N.check(self._L.cf_step_item_reduce(self._h, int(piece)), "cf_step_item_reduce")

    def item_piece_rows(self, piece, n_pieces):
        """Item rows [row0, row1) of piece `piece` of n_pieces."""
        r0, r1 = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(self._L.cf_item_piece_rows(self._h, int(piece), int(n_pieces), ctypes.byref(r0),
                                           ctypes.byref(r1)), "cf_item_piece_rows")
        return int(r0.value), int(r1.value)

    def step_items(self):
        N.check(self._L.cf_step_items(self._h), "cf_step_items")

    def step_local_draw(self, batch_size):
        N.check(self._L.cf_step_local_draw(self._h, int(batch_size)), "cf_step_local_draw")

    # item-range ownership (reduce-scatter -> owner Adagrad -> all-gather)
    def bind_item_grad_split(self, grad_items_ptr, n_grad_items, grad_bias_ptr=None, n_grad_bias=0):
        v = ctypes.c_void_p
        N.check(self._L.cf_bind_item_grad_split(self._h, v(grad_items_ptr), int(n_grad_items),
                                                v(grad_bias_ptr or None), int(n_grad_bias)),
                "cf_bind_item_grad_split")

    def clear_item_grad(self):
        N.check(self._L.cf_clear_item_grad(self._h), "cf_clear_item_grad")

    def step_items_range(self, row0, row1, grad, grad_bias=None):
        """grad / grad_bias: device pointers or torch device tensors."""
        v = ctypes.c_void_p
        p = lambda t: (t.data_ptr() if hasattr(t, "data_ptr") else t) or None  # noqa: E731
        N.check(self._L.cf_step_items_range(self._h, int(row0), int(row1), v(p(grad)),
                                            v(p(grad_bias))), "cf_step_items_range")

    def bind_table(self, name, device_ptr, n_elems):
        """Caller device memory (e.g. a padded torch tensor) as the storage
        of an item-side table; None returns it to engine-owned memory."""
        N.check(self._L.cf_bind_table(self._h, N.TABLES[name], ctypes.c_void_p(device_ptr or None),
                                      int(n_elems)), "cf_bind_table(%s)" % name)

    # ---- user sharding + GBPR group exchange (include/cf_engine.h) --------------
    def set_shard(self, world, rank, bounds):
        b = np.ascontiguousarray(bounds, dtype=np.int64)
        N.check(self._L.cf_set_shard(self._h, int(world), int(rank), _ptr(b, ctypes.c_int64)),
                "cf_set_shard")

    def set_group_source(self, indptr_t, indices_t):
        ip = np.ascontiguousarray(indptr_t, dtype=np.int64)
        ix = np.ascontiguousarray(indices_t, dtype=np.int32)
        N.check(self._L.cf_set_group_source(self._h, _ptr(ip, ctypes.c_int64),
                                            _ptr(ix, ctypes.c_int32), int(ix.shape[0])),
                "cf_set_group_source")

    def bind_exchange(self, send_ids, rows, grads, send_cap, recv_ids, serve_rows, serve_grads,
                      recv_cap):
        v = ctypes.c_void_p
        N.check(self._L.cf_bind_exchange(self._h, v(send_ids), v(rows), v(grads), int(send_cap),
                                         v(recv_ids), v(serve_rows), v(serve_grads), int(recv_cap)),
                "cf_bind_exchange")

    def xchg_begin(self, world, batch_size=None, pairs=None, negs=None, groups=None):
        """Draw (or take) the batch, pack remote group members by owner;
        returns the number of ids sent to each rank (groups: GLOBAL ids)."""
        counts = np.zeros(int(world), dtype=np.int32)
        cp = _ptr(counts, ctypes.c_int32)
        if pairs is None:
            N.check(self._L.cf_xchg_begin(self._h, int(batch_size), None, None, None, cp),
                    "cf_xchg_begin")
        else:
            B, pairs, negs, gp, _keep = self._batch(pairs, negs, groups)
            N.check(self._L.cf_xchg_begin(self._h, B, _arg(pairs, ctypes.c_int32),
                                          _arg(negs, ctypes.c_int32), gp, cp), "cf_xchg_begin")
        return counts

    def xchg_draw(self, batch_size, send_counts_dev_ptr):
        """Draw + pack the NEXT exchange batch (no host sync); its per-owner
        counts go to the device int32 [2, world] buffer at row `half`, its
        ids to half `half` of send_ids.  Returns half."""
        h = ctypes.c_int32(0)
        N.check(self._L.cf_xchg_draw(self._h, int(batch_size), ctypes.c_void_p(send_counts_dev_ptr),
                                     ctypes.byref(h)), "cf_xchg_draw")
        return int(h.value)

    def xchg_adopt(self, batch_size):
        """Take the batch drawn ahead as this step's.  False (CF_EAGAIN) when
        none of that size is pending -- a batch drawn at another size is
        discarded by the engine (counts cleared, sampler rewound)."""
        st = self._L.cf_xchg_adopt(self._h, int(batch_size))
        if st == N.CF_EAGAIN:
            return False
        N.check(st, "cf_xchg_adopt")
        return True

    def xchg_serve(self, n_recv):
        N.check(self._L.cf_xchg_serve(self._h, int(n_recv)), "cf_xchg_serve")

    def xchg_grad(self):
        N.check(self._L.cf_xchg_grad(self._h), "cf_xchg_grad")

    def xchg_grad_part(self, part):
        N.check(self._L.cf_xchg_grad_part(self._h, int(part)), "cf_xchg_grad_part")

    def xchg_finish_items(self):
        N.check(self._L.cf_xchg_finish_items(self._h), "cf_xchg_finish_items")

    def xchg_finish(self, n_recv):
        N.check(self._L.cf_xchg_finish(self._h, int(n_recv)), "cf_xchg_finish")

    def take_loss(self):
        v = ctypes.c_double(0.0)
        N.check(self._L.cf_take_loss(self._h, ctypes.byref(v)), "cf_take_loss")
        return float(v.value)

    # ---- evaluation -------------------------------------------------------------
    def score_topk(self, users, k, exclude_train=True, return_values=False, item_mask=None):
        """Top-k items per user (cf_score_topk_ex): exclude_train drops each
        user's train items (the reference's __recommend filter), item_mask
        (bool / uint8 [n_items], numpy or a torch device tensor) drops the
        flagged items for every user on top."""
        mp, mkeep = None, None
        if item_mask is not None:
            if _is_dev(item_mask):
                import torch
                mkeep, _ = _dev(item_mask.reshape(-1), torch.uint8, ctypes.c_uint8)
                mp = ctypes.c_void_p(mkeep.data_ptr())
            else:
                mkeep = np.ascontiguousarray(item_mask, dtype=np.uint8).reshape(-1)
                mp = ctypes.c_void_p(mkeep.ctypes.data)
            if mkeep.shape[0] != self.n_items:
                raise ValueError("item_mask must have n_items entries")
        if _is_dev(users):   # device ids in, device results out
            import torch
            u, up = _dev(users.reshape(-1), torch.int32, ctypes.c_int32)
            n = u.shape[0]
            idx = torch.empty((n, int(k)), dtype=torch.int32, device=u.device)
            val = torch.empty((n, int(k)), dtype=torch.float32, device=u.device) if return_values else None
            N.check(self._L.cf_score_topk_ex(
                self._h, up, n, int(k), 1 if exclude_train else 0, mp,
                ctypes.cast(idx.data_ptr(), ctypes.POINTER(ctypes.c_int32)),
                ctypes.cast(val.data_ptr(), ctypes.POINTER(ctypes.c_float)) if return_values else None),
                "cf_score_topk_ex")
            return (idx, val) if return_values else idx
        users = _i32(users).reshape(-1)
        n = users.shape[0]
        idx = np.empty((n, int(k)), dtype=np.int32)
        val = np.empty((n, int(k)), dtype=np.float32) if return_values else None
        N.check(self._L.cf_score_topk_ex(self._h, _ptr(users, ctypes.c_int32), n, int(k),
                                         1 if exclude_train else 0, mp, _ptr(idx, ctypes.c_int32),
                                         _ptr(val, ctypes.c_float) if return_values else None),
                "cf_score_topk_ex")
        return (idx, val) if return_values else idx

    def recommend(self, users, k, mask=None):
        """cf_score_topk with SURVEY 8(b)'s mask_or_NULL: None = exclude each
        user's train items; a uint8 [n_items] mask = exactly those items."""
        users = _i32(users).reshape(-1)
        n = users.shape[0]
        idx = np.empty((n, int(k)), dtype=np.int32)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8).reshape(-1)
        if m is not None and m.shape[0] != self.n_items:
            raise ValueError("mask must have n_items entries")
        N.check(self._L.cf_score_topk(self._h, _ptr(users, ctypes.c_int32), n, int(k),
                                      None if m is None else ctypes.c_void_p(m.ctypes.data),
                                      _ptr(idx, ctypes.c_int32), None), "cf_score_topk")
        return idx

    PATH_FLAGS = {"phased": 1, "pos_sort": 2, "item_records": 4, "deterministic": 8, "dense_items": 16,
                  "lds": 32, "sorted_batches": 64}

    def step_path(self, batch_size):
        """The kernel path a step of ``batch_size`` pairs takes now
        (cf_step_path): (flags, {name: bool, ..., "pipeline": n})."""
        f = ctypes.c_int32(0)
        N.check(self._L.cf_step_path(self._h, int(batch_size), ctypes.byref(f)), "cf_step_path")
        v = int(f.value)
        out = {k: bool(v & m) for k, m in self.PATH_FLAGS.items()}
        out["pipeline"] = (v >> 8) & 3
        return v, out

    def set_option(self, name, value):
        N.check(self._L.cf_set_option(self._h, name.encode(), int(value)), "cf_set_option(%s)" % name)

    # ---- measurement -------------------------------------------------------------
    def profile(self, on=True):
        N.check(self._L.cf_profile_enable(self._h, 1 if on else 0), "cf_profile_enable")

    def profile_read(self, kernel):
        ms, n = ctypes.c_double(0.0), ctypes.c_int64(0)
        N.check(self._L.cf_profile_read(self._h, N.KERNELS[kernel], ctypes.byref(ms),
                                        ctypes.byref(n)), "cf_profile_read")
        return float(ms.value), int(n.value)

    def profile_reset(self):
        N.check(self._L.cf_profile_reset(self._h), "cf_profile_reset")


def synth_degrees(n_users, mean_degree, seed):
    """Global indptr (int64, n_users+1) of the synthetic graph's degrees."""
    L = N.lib()
    indptr = np.empty(int(n_users) + 1, dtype=np.int64)
    N.check(L.cf_synth_degrees(int(n_users), float(mean_degree), int(seed), 0, int(n_users),
                               _ptr(indptr, ctypes.c_int64)), "cf_synth_degrees")
    return indptr


def synth_graph(n_users, n_items, mean_degree, zipf_s, seed, u_begin=0, u_end=None, n_threads=0):
    """CSR (indptr int64, indices int32) of users [u_begin, u_end) of the
    synthetic implicit-feedback graph; host-side, deterministic."""
    L = N.lib()
    if u_end is None:
        u_end = n_users
    nu = int(u_end) - int(u_begin)
    indptr = np.empty(nu + 1, dtype=np.int64)
    N.check(L.cf_synth_degrees(int(n_users), float(mean_degree), int(seed), int(u_begin),
                               int(u_end), _ptr(indptr, ctypes.c_int64)), "cf_synth_degrees")
    indices = np.empty(int(indptr[-1]), dtype=np.int32)
    N.check(L.cf_synth_items(int(n_items), float(zipf_s), int(seed), int(u_begin), int(u_end),
                             _ptr(indptr, ctypes.c_int64), _ptr(indices, ctypes.c_int32),
                             int(n_threads)), "cf_synth_items")
    return indptr, indices


def synth_item_users(n_users, n_items, mean_degree, zipf_s, seed, n_threads=0):
    """Item -> user CSR (indptr int64 [n_items+1], indices int32) of the whole
    synthetic graph, users of each item ascending (cf_synth_item_users): the
    GBPR group source of a user-sharded engine, built natively."""
    L = N.lib()
    degs = synth_degrees(n_users, mean_degree, seed)
    nnz = int(degs[-1])
    del degs
    indptr_t = np.empty(int(n_items) + 1, dtype=np.int64)
    indices_t = np.empty(nnz, dtype=np.int32)
    N.check(L.cf_synth_item_users(int(n_users), int(n_items), float(mean_degree), float(zipf_s),
                                  int(seed), _ptr(indptr_t, ctypes.c_int64),
                                  _ptr(indices_t, ctypes.c_int32), int(n_threads)),
            "cf_synth_item_users")
    return indptr_t, indices_t
