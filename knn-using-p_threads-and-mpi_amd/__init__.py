"""Python host mirror of the MI355X KNN path (ctypes over libknn_amd.so).

The product is the C ABI in ``include/knn_amd.h`` (plus the reference-compatible C++
API in ``include/knn_arff.hpp``); this module binds it for the tests and ``bench.py``.
Names follow the reference (srna99/KNN-using-p_threads-and-MPI):

* ``KNN(train, test, k)``                      main.cpp:25      -> int32 predictions
* ``KNN_range(train, test, k, start, end)``    mpi.cpp:26 / multi-thread.cpp:37
* ``computeConfusionMatrix(pred, labels, C)``  main.cpp:87
* ``computeAccuracy(cm, n)``                   main.cpp:102
* ``read_arff(path)``                          libarff ArffParser::parse (arff_parser.cpp:23)
* ``shard_range(n, world, rank)``              multi-thread.cpp:154-158 / mpi.cpp:141-170
* ``train_sharded_predict(...)``               train-sharded KNN over ranks:
  per-shard exact top-k -> all-to-all of neighbour lists -> merge + vote

Features are fp32 or bf16.  Host bf16 arrays are numpy ``uint16`` holding bf16 bits
(``to_bf16_bits`` / ``bf16_bits_to_f32``); device tensors are ``torch.bfloat16``.

There is no CPU fallback: if ``libknn_amd.so`` is missing or no gfx950 device is
visible, calls raise ``KnnError``.
"""
import ctypes
import os
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# KNN_AMD_LIB overrides the library (A/B runs of alternative builds)
LIB_PATH = os.environ.get("KNN_AMD_LIB") or os.path.join(_HERE, "libknn_amd.so")

KNN_OK, KNN_EINVAL, KNN_ENOMEM, KNN_EHIP, KNN_ERANGE, KNN_ENODEV, KNN_EIO, KNN_ERCCL = range(8)
STATUS_NAMES = {0: "KNN_OK", 1: "KNN_EINVAL", 2: "KNN_ENOMEM", 3: "KNN_EHIP", 4: "KNN_ERANGE",
                5: "KNN_ENODEV", 6: "KNN_EIO", 7: "KNN_ERCCL"}
KNN_COMM_ID_BYTES = 128
KNN_F32, KNN_BF16 = 0, 1
ALGOS = {"auto": 0, "direct": 1, "gemm": 2, "gemm_split": 3, "gemm_bf16": 4, "direct_scan": 5}
FILTER_OPERANDS = {-1: None, 0: "f32", 1: "bf16", 2: "bf16x3 split", 3: "bf16 rounded"}


class KnnError(RuntimeError):
    def __init__(self, status, msg=""):
        self.status = status
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")


KNN_OPT_CACHE_TRAIN = 1
KNN_OPT_CACHE_TRAIN_DEVICE = 2
# contexts holding a cached device train tensor: Context.generate invalidates every one whose
# tensor shares bytes with what it writes (a slice, a view, another context's call)
_caching_contexts = weakref.WeakSet()


def _byte_span(t):
    """[first, last) device byte addresses a strided tensor covers (empty: (p, p))."""
    p = t.data_ptr()
    if t.numel() == 0:
        return p, p
    hi = sum((n - 1) * st for n, st in zip(t.shape, t.stride())) + 1
    return p, p + hi * t.element_size()


class knn_opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("algo", ctypes.c_int32),
                ("train_splits", ctypes.c_int32), ("profile", ctypes.c_int32), ("flags", ctypes.c_int32)]


class knn_dataset(ctypes.Structure):
    _fields_ = [("feat", ctypes.c_void_p), ("labels", ctypes.c_void_p), ("n", ctypes.c_int64),
                ("d", ctypes.c_int32), ("ld", ctypes.c_int32), ("dtype", ctypes.c_int32)]


_lib = None


def load_library(path=LIB_PATH):
    """Load libknn_amd.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise KnnError(KNN_ENODEV, f"{path} not built: run `make -C {_HERE}` "
                                   "(or __graft_entry__.build())")
    # The torch wheel bundles its own ROCm runtime whose libamdhip64 has the same SONAME
    # (libamdhip64.so.7) as /opt/rocm's.  Loading torch first makes this library bind to
    # that already-loaded runtime, so a process never holds two HIP/HSA runtimes (which
    # leaves whichever initialises second without a device).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    P, I32, I64, F = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float
    DS = ctypes.POINTER(knn_dataset)
    sig = {
        "knn_version": (I32, []),
        "knn_build_id": (ctypes.c_char_p, []),
        "knn_create": (I32, [ctypes.POINTER(P), ctypes.POINTER(knn_opts)]),
        "knn_destroy": (None, [P]),
        "knn_last_error": (ctypes.c_char_p, [P]),
        "knn_predict": (I32, [P, DS, DS, I32, I32, I64, I64, P, P, P]),
        "knn_predict_device": (I32, [P, DS, DS, I32, I32, P, P, P, P]),
        "knn_shard_topk_device": (I32, [P, DS, DS, I32, I32, I64, P, P]),
        "knn_merge_vote_device": (I32, [P, I32, I64, I32, I32, P, P, P, P, P]),
        "knn_stage_times": (I32, [P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(F), I32]),
        "knn_last_stats": (I32, [P, ctypes.POINTER(I64), I32]),
        "knn_generate": (I32, [P, P, P, I64, I64, I32, I32, I32, I32, ctypes.c_uint64,
                               ctypes.c_uint32, I32, P]),
        "knn_mfma_probe_bf16": (I32, [P, P, P, I32, P, P]),
        "knn_set_generation": (I32, [P, ctypes.c_uint64]),
        "knn_comm_unique_id": (I32, [P]),
        "knn_comm_create": (I32, [P, P, I32, I32, ctypes.POINTER(P)]),
        "knn_comm_destroy": (None, [P]),
        "knn_comm_count": (I32, [P, ctypes.POINTER(I32)]),
        "knn_comm_broken": (I32, [P, ctypes.POINTER(I32)]),
        "knn_comm_set_exchange": (I32, [P, I64, I32]),
        "knn_predict_train_sharded": (I32, [P, P, DS, I64, DS, I32, I32, P, P, P, P]),
        "knn_shard_range": (I32, [I64, I32, I32, ctypes.POINTER(I64), ctypes.POINTER(I64)]),
        "knn_shard_policy": (I32, [I64, I64, I32, I32, I32, I64, ctypes.POINTER(I32)]),
        "knn_exchange_layout": (I32, [I64, I32, I32, I32, P, P, P, P]),
        "knn_alloc_pinned": (I32, [ctypes.c_size_t, ctypes.POINTER(P)]),
        "knn_free_pinned": (None, [P]),
        "knn_confusion_matrix": (I32, [P, P, I64, I32, P]),
        "knn_confusion_matrix_device": (I32, [P, P, P, I64, I32, P, P, P]),
        "knn_accuracy": (F, [P, I32, I64]),
        "knn_arff_open": (I32, [ctypes.c_char_p, ctypes.POINTER(P), ctypes.c_char_p, I32]),
        "knn_arff_shape": (None, [P, ctypes.POINTER(I64), ctypes.POINTER(I32), ctypes.POINTER(I32)]),
        "knn_arff_copy": (I32, [P, P, I32, P]),
        "knn_arff_close": (None, [P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def to_bf16_bits(x):
    """float32 array -> uint16 bf16 bits (round to nearest even; exact for bf16 values)."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def bf16_bits_to_f32(b):
    """uint16 bf16 bits -> the exactly widened float32 values."""
    return (np.ascontiguousarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32)


def _dataset(feat, labels=None):
    """numpy features (float32, or uint16 = bf16 bits) -> knn_dataset (+ arrays to keep alive)."""
    if isinstance(feat, np.ndarray) and feat.dtype == np.uint16:
        feat, dtype = np.ascontiguousarray(feat), KNN_BF16
    else:
        feat, dtype = np.ascontiguousarray(feat, dtype=np.float32), KNN_F32
    if feat.ndim != 2:
        raise KnnError(KNN_EINVAL, "features must be 2-D [n][d]")
    lab = None if labels is None else np.ascontiguousarray(labels, dtype=np.int32)
    ds = knn_dataset(feat.ctypes.data, None if lab is None else lab.ctypes.data, feat.shape[0],
                     feat.shape[1], feat.shape[1], dtype)
    return ds, (feat, lab)  # keep the arrays alive


def _tensor_dtype(t):
    import torch
    if t.dtype == torch.bfloat16:
        return KNN_BF16
    if t.dtype == torch.float32:
        return KNN_F32
    raise KnnError(KNN_EINVAL, f"features must be float32 or bfloat16, got {t.dtype}")


def _check_tensor(t, name, dtype, n=None):
    """A device output/label tensor: contiguous, of the element type the C ABI reads."""
    import torch
    if t.dtype != dtype:
        raise KnnError(KNN_EINVAL, f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise KnnError(KNN_EINVAL, f"{name} must be contiguous")
    if n is not None and t.numel() < n:
        raise KnnError(KNN_EINVAL, f"{name} holds {t.numel()} elements, needs {n}")
    return t


def _device_dataset(feat, labels=None, d=None):
    """A [n][ld] device tensor (unit stride along features; ld = its row stride) and its
    int32 labels -> knn_dataset.  Views such as x[:, :64] of a wider tensor are accepted
    (ld = the parent's row stride); anything with non-unit feature stride is rejected."""
    import torch
    if feat.dim() != 2:
        raise KnnError(KNN_EINVAL, "features must be a 2-D [n][ld] tensor")
    if feat.shape[0] > 1 and feat.stride(1) != 1:
        raise KnnError(KNN_EINVAL, "features must have unit stride along the feature axis")
    ld = feat.stride(0) if feat.shape[0] > 1 else feat.shape[1]
    d = feat.shape[1] if d is None else d
    if d > feat.shape[1]:
        raise KnnError(KNN_EINVAL, f"d={d} exceeds the tensor's {feat.shape[1]} columns")
    if labels is not None:
        _check_tensor(labels, "labels", torch.int32, feat.shape[0])
    return knn_dataset(feat.data_ptr(), None if labels is None else labels.data_ptr(), feat.shape[0], d,
                       ld, _tensor_dtype(feat))


def _stream_arg(stream, tensor):
    """The HIP stream a device call is enqueued on: the caller's, else torch's current stream
    of the tensor's device -- so the call is ordered after the torch work that produced its
    inputs (a copy, a dtype conversion, a clone) and before the torch work that reads its
    outputs, with no extra synchronisation."""
    if stream is None and tensor is not None and getattr(tensor, "is_cuda", False):
        import torch
        # (the raw handle: 0.08 us per call against 1.9 for a torch.cuda.Stream object, on a
        # ~0.1 ms config-L call; scripts/diag_call_overhead.py)
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        stream = raw(tensor.device.index) if raw is not None else torch.cuda.current_stream(tensor.device).cuda_stream
    return None if stream is None else ctypes.c_void_p(stream)


def _outputs(nq, k, pred=None, dist=None, idx=None):
    """Type/shape checks of device outputs (pred int32 [nq], dist float32 / idx int32 [nq][k])."""
    import torch
    if pred is not None:
        _check_tensor(pred, "pred", torch.int32, nq)
    if dist is not None:
        _check_tensor(dist, "dist", torch.float32, nq * k)
    if idx is not None:
        _check_tensor(idx, "idx", torch.int32, nq * k)


def shard_range(n, world, rank):
    """Contiguous split with the remainder on the last worker (multi-thread.cpp:154-158,
    mpi.cpp:141-170): worker w < world-1 gets [w*(n//world), (w+1)*(n//world))."""
    per, left = divmod(n, world)
    start = rank * per
    return start, start + per + (left if rank == world - 1 else 0)


def rank_queries(n_query, world, rank, scaling):
    """Query rows [q0, q0+nq) a rank owns.  "strong": the reference's split of a fixed
    test set (shard_range).  "weak": every rank owns n_query rows of its own,
    rank r taking global rows [r*n_query, (r+1)*n_query)."""
    if scaling == "weak":
        return rank * n_query, n_query
    q0, q1 = shard_range(n_query, world, rank)
    return q0, q1 - q0


def gather_predictions(pred_local, q0, n_total, world, rank, group=None):
    """Rank 0 receives every rank's predictions at their global offsets -- the
    reference's MPI_Gatherv (mpi.cpp:177-186) -- over torch.distributed (any backend).
    Returns the full int32 vector on rank 0, None elsewhere."""
    import torch.distributed as dist
    pred_local = np.ascontiguousarray(pred_local, np.int32)
    parts = [None] * world if rank == 0 else None
    dist.gather_object((int(q0), pred_local), parts, dst=0, group=group)
    if rank != 0:
        return None
    out = np.full(n_total, -1, np.int32)
    for off, p in parts:
        out[off:off + len(p)] = p
    return out


def exchange_shard_lists(rec, n_query, world, rank, group=None):
    """The train-sharded exchange: every rank holds its shard's neighbour
    lists for ALL queries, rec [n_query][3][k]; rank r owns queries shard_range(n_query,
    world, r) (the reference's split, mpi.cpp:141-170).  One all-to-all (RCCL over xGMI on
    the GPU node; any torch.distributed backend works) hands each rank the lists of its
    own queries from every shard: returns [world][nq_r][3][k] (source rank order = shard
    order = global index order) and this rank's query range (q0, q1)."""
    import torch
    import torch.distributed as dist
    k3 = rec.shape[1] * rec.shape[2]
    spans = [shard_range(n_query, world, r) for r in range(world)]
    q0, q1 = spans[rank]
    send = [(b - a) * k3 for a, b in spans]          # to rank r: its query rows
    recv = [(q1 - q0) * k3] * world                   # from every rank: my query rows
    out = torch.empty((world, q1 - q0) + tuple(rec.shape[1:]), dtype=rec.dtype, device=rec.device)
    if world == 1:
        out[0].copy_(rec)
    else:
        dist.all_to_all_single(out.view(-1), rec.contiguous().view(-1), recv, send, group=group)
    return out, (q0, q1)


def train_sharded_predict(ctx, train_shard, labels_shard, idx_base, test, k, num_classes, world, rank,
                          group=None, dist_out=None, idx_out=None, stream=None):
    """KNN with the train set sharded over ranks: this rank's
    shard (global rows [idx_base, idx_base + n)) against every query -> exchange ->
    merge + vote for the queries this rank owns.  Returns (pred [nq_r] int32 device
    tensor, (q0, q1)).  Bit-identical to the reference's serial KNN over the whole set."""
    import torch
    nq = test.shape[0]
    if stream is None and test.is_cuda:
        # one stream for topk -> all-to-all -> merge (the collective is ordered on torch's
        # current stream, so the merge must be too)
        stream = torch.cuda.current_stream(test.device).cuda_stream
    rec = torch.empty((nq, 3, k), dtype=torch.int32, device=test.device)
    ctx.shard_topk_device(train_shard, labels_shard, test, k, num_classes, idx_base, rec, stream=stream)
    lists, (q0, q1) = exchange_shard_lists(rec, nq, world, rank, group)
    del rec
    pred = torch.empty(q1 - q0, dtype=torch.int32, device=test.device)
    ctx.merge_vote_device(lists, k, num_classes, pred, dist_out, idx_out, stream=stream)
    return pred, (q0, q1)


class Context:
    """One device, one HIP stream (knn_create / knn_destroy)."""

    def __init__(self, device=0, algo="auto", train_splits=0, profile=False, cache_train=False):
        self.lib = load_library()
        # profile: False/0 off, True/1 per-stage HIP events, 2 = also count filter candidates,
        # 3 = events around the dominant stages only (filter, rescore, ...: knn_amd.h)
        # cache_train: predict() keeps the device copy of train across calls (KNN_OPT_CACHE_TRAIN)
        # and the device calls keep the operands derived from the caller's train tensor
        # (KNN_OPT_CACHE_TRAIN_DEVICE): this wrapper bumps the generation on every write it can see
        opts = knn_opts(device, ALGOS[algo], train_splits, int(profile),
                        KNN_OPT_CACHE_TRAIN | KNN_OPT_CACHE_TRAIN_DEVICE if cache_train else 0)
        self.cache_train = bool(cache_train)
        # the arrays whose addresses key the library's train cache (knn_predict): held until
        # the next call replaces them, so no later array can be allocated at a cached address
        # (_dataset copies inputs of another dtype or layout into temporaries)
        self._train_key = None
        # device calls under cache_train: the train tensor whose filter operands the library
        # keeps (knn_predict_device / knn_shard_topk_device), and its torch version counter --
        # a different tensor or an in-place write bumps the library's generation, and holding
        # the tensor keeps its address from being reused while it is cached
        self._dev_train = None
        self._generation = 0
        self.device = int(device)
        h = ctypes.c_void_p()
        st = self.lib.knn_create(ctypes.byref(h), ctypes.byref(opts))
        if st != KNN_OK:
            raise KnnError(st, f"knn_create(device={device}) failed")
        self.h = h

    def _check(self, st):
        if st != KNN_OK:
            raise KnnError(st, self.lib.knn_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            self.lib.knn_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def predict(self, train_feat, train_labels, test_feat, k, num_classes=None, q_begin=0,
                q_end=None, topk=False):
        """Host arrays in, host arrays out (knn_predict)."""
        tr, keep1 = _dataset(train_feat, train_labels)
        te, keep2 = _dataset(test_feat)
        if num_classes is None:
            num_classes = int(keep1[1].max()) + 1 if keep1[1].size else 1
        if q_end is None:
            q_end = te.n
        nq = q_end - q_begin
        pred = np.zeros(max(nq, 0), np.int32)
        dist = np.zeros((max(nq, 0), k), np.float32) if topk else None
        idx = np.zeros((max(nq, 0), k), np.int32) if topk else None
        if self.cache_train:
            self._train_key = keep1
        self._check(self.lib.knn_predict(self.h, ctypes.byref(tr), ctypes.byref(te), k, num_classes,
                                         q_begin, q_end, _ptr(pred), _ptr(dist), _ptr(idx)))
        return (pred, dist, idx) if topk else pred

    def _on_device(self, tensor):
        """The tensor lives on this context's device (a call on another device's stream fails
        inside HIP with an unhelpful error)."""
        if tensor is not None and getattr(tensor, "is_cuda", False) and tensor.device.index != self.device:
            raise KnnError(KNN_EINVAL, f"tensor on cuda:{tensor.device.index}, context on device {self.device}")

    def _stream(self, stream, tensor):
        """_stream_arg, after _on_device."""
        self._on_device(tensor)
        return _stream_arg(stream, tensor)

    def _note_train(self, train):
        """cache_train: bump the generation when the train tensor is another one or was written
        in place since the last device call (torch's version counter)."""
        if not self.cache_train:
            return
        key = (train.data_ptr(), tuple(train.shape), train._version)
        if self._dev_train is None or self._dev_train[0] is not train or self._dev_train[1] != key:
            self.set_generation(self._generation + 1)
            self._dev_train = (train, key)
            _caching_contexts.add(self)

    def _invalidate_overlap(self, span):
        """The cached train tensor shares bytes with [span): the next device call bumps the
        generation (the write did not go through torch, so its version counter did not move)."""
        if self._dev_train is not None:
            a, b = _byte_span(self._dev_train[0])
            if a < span[1] and span[0] < b:
                self._dev_train = None

    def predict_device(self, train, labels, test, k, num_classes, pred, dist=None, idx=None,
                       stream=None, d=None):
        """Device tensors (torch, on this context's device) in and out (knn_predict_device).
        train/test: [n][ld] float32 contiguous; labels/pred/idx int32; dist float32.
        With cache_train the train-side filter operands are kept across calls on the same,
        unmodified train tensor (rewrites through torch are seen; after writing it by other
        means call set_generation)."""
        self._on_device(train)
        self._note_train(train)
        tr = _device_dataset(train, labels, d)
        te = _device_dataset(test, None, d)
        _outputs(te.n, k, pred, dist, idx)
        self._check(self.lib.knn_predict_device(
            self.h, ctypes.byref(tr), ctypes.byref(te), k, num_classes, pred.data_ptr(),
            None if dist is None else dist.data_ptr(), None if idx is None else idx.data_ptr(),
            self._stream(stream, test)))

    def shard_topk_device(self, train, labels, test, k, num_classes, idx_base, rec, stream=None, d=None):
        """Exact k nearest rows of one train shard for every query (knn_shard_topk_device).
        rec: int32 device tensor [nq][3][k] <- (dist bits, idx_base + row, label), ascending."""
        self._on_device(train)
        self._note_train(train)
        tr = _device_dataset(train, labels, d)
        te = _device_dataset(test, None, d)
        if tuple(rec.shape) != (test.shape[0], 3, k):
            raise KnnError(KNN_EINVAL, f"rec must be [{test.shape[0]}, 3, {k}]")
        import torch
        _check_tensor(rec, "rec", torch.int32)
        self._check(self.lib.knn_shard_topk_device(
            self.h, ctypes.byref(tr), ctypes.byref(te), k, num_classes, idx_base, rec.data_ptr(),
            self._stream(stream, test)))

    def merge_vote_device(self, rec, k, num_classes, pred, dist=None, idx=None, stream=None):
        """Merge nsrc per-shard neighbour lists rec [nsrc][nq][3][k] and vote (knn_merge_vote_device)."""
        nsrc, nq = rec.shape[0], rec.shape[1]
        if tuple(rec.shape[2:]) != (3, k) or pred.shape[0] != nq:
            raise KnnError(KNN_EINVAL, "rec must be [nsrc][nq][3][k] and pred [nq]")
        import torch
        _check_tensor(rec, "rec", torch.int32)
        _outputs(nq, k, pred, dist, idx)
        self._check(self.lib.knn_merge_vote_device(
            self.h, nsrc, nq, k, num_classes, rec.data_ptr(), pred.data_ptr(),
            None if dist is None else dist.data_ptr(), None if idx is None else idx.data_ptr(),
            self._stream(stream, rec)))

    def generate(self, feat, labels, row0, d, kind, seed, stream_id, num_classes, dtype=None,
                 stream=None):
        """Fill a device tensor [n][ld] (and labels) with the synthetic rows of SURVEY.md 8d.
        kind 0 / 1: uniform fp32 grid / bf16-exact values; 2 / 3: the same clustered (the row's
        class centroid + noise: labels carry signal).  A bfloat16 tensor receives bf16 bits
        (kinds 1 and 3: bf16-exact values)."""
        dtype = _tensor_dtype(feat) if dtype is None else dtype
        self._check(self.lib.knn_generate(
            self.h, feat.data_ptr(), None if labels is None else labels.data_ptr(), row0,
            feat.shape[0], d, feat.shape[1], dtype, kind, seed, stream_id, num_classes,
            self._stream(stream, feat)))
        # written behind torch's back: every context caching a train tensor that shares bytes with
        # feat (feat itself, a slice or view of it, a tensor feat is a view of) bumps its
        # generation at its next call
        span = _byte_span(feat)
        for c in list(_caching_contexts):
            c._invalidate_overlap(span)

    def confusion_matrix_device(self, pred, labels, num_classes, cm=None, stream=None):
        """computeConfusionMatrix / computeAccuracy (main.cpp:87-112) on device tensors:
        returns (cm int32 [C][C] device tensor, accuracy as the reference's float)."""
        import torch
        _check_tensor(pred, "pred", torch.int32)
        _check_tensor(labels, "labels", torch.int32, pred.shape[0])
        if cm is None:
            cm = torch.empty((num_classes, num_classes), dtype=torch.int32, device=pred.device)
        corr = torch.zeros(1, dtype=torch.int64, device=pred.device)
        self._check(self.lib.knn_confusion_matrix_device(
            self.h, pred.data_ptr(), labels.data_ptr(), pred.shape[0], num_classes, cm.data_ptr(),
            corr.data_ptr(), self._stream(stream, pred)))
        n = pred.shape[0]
        return cm, float(np.float32(int(corr.item())) / np.float32(n)) if n else float("nan")

    def mfma_probe_bf16(self, a, b, stream=None):
        """The bf16 filter's MFMA chain on device operands a, b: [32][K] torch.bfloat16
        (K % 16 == 0) -> float32 [32][32] = a @ b.T as v_mfma_f32_32x32x16_bf16 sums it."""
        import torch
        if a.shape != b.shape or a.dim() != 2 or a.shape[0] != 32 or a.dtype != torch.bfloat16:
            raise KnnError(KNN_EINVAL, "a, b must be [32][K] bfloat16")
        a, b = a.contiguous(), b.contiguous()
        out = torch.empty((32, 32), dtype=torch.float32, device=a.device)
        self._check(self.lib.knn_mfma_probe_bf16(self.h, a.data_ptr(), b.data_ptr(), a.shape[1], out.data_ptr(),
                                                 self._stream(stream, a)))
        return out

    def set_generation(self, generation):
        """Invalidate cached train uploads and train-side filter operands (knn_set_generation)."""
        self._check(self.lib.knn_set_generation(self.h, generation))
        self._generation = int(generation)

    def stage_times(self):
        names = (ctypes.c_char_p * 256)()
        ms = (ctypes.c_float * 256)()
        n = self.lib.knn_stage_times(self.h, names, ms, 256)
        out = {}
        for i in range(n):
            key = names[i].decode()
            out[key] = out.get(key, 0.0) + ms[i]
        return out

    def stats(self):
        v = (ctypes.c_int64 * 11)()
        self.lib.knn_last_stats(self.h, v, 11)
        return {"candidates": v[0], "fallback_queries": v[1], "train_segments": v[2],
                "filter_operands": FILTER_OPERANDS.get(v[3], v[3]), "rerun_split": bool(v[4]),
                "fused_norm": bool(v[5]), "h2d_train_bytes": v[6], "h2d_query_bytes": v[7],
                "train_operands_cached": bool(v[8]), "filter_mfma": v[9],
                "queries_per_wave": v[10]}


def comm_unique_id():
    """knn_comm_unique_id: 128 bytes to hand to every rank (the caller's bootstrap)."""
    lib = load_library()
    buf = ctypes.create_string_buffer(KNN_COMM_ID_BYTES)
    st = lib.knn_comm_unique_id(buf)
    if st != KNN_OK:
        raise KnnError(st, "knn_comm_unique_id")
    return buf.raw


def build_id():
    """(id baked into the loaded libknn_amd.so, id of the sources beside it): equal when the
    library was built from this tree (build_id.py)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("knn_amd_build_id", os.path.join(_HERE, "build_id.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return load_library().knn_build_id().decode(), mod.compute()


def shard_range_c(n, world, rank):
    """knn_shard_range (the C ABI's copy of shard_range, used by knn_predict_train_sharded)."""
    lib = load_library()
    a, b = ctypes.c_int64(), ctypes.c_int64()
    st = lib.knn_shard_range(n, world, rank, ctypes.byref(a), ctypes.byref(b))
    if st != KNN_OK:
        raise KnnError(st, "knn_shard_range")
    return a.value, b.value


def shard_policy(n_train, n_query, d, dtype, world, hbm_bytes=0):
    """knn_shard_policy: "test" (queries split, train replicated) or "train" (train split,
    per-shard top-k exchanged and merged) for a world-GPU run.  dtype: "f32" or "bf16"."""
    lib = load_library()
    p = ctypes.c_int32()
    st = lib.knn_shard_policy(n_train, n_query, d, KNN_BF16 if dtype == "bf16" else KNN_F32, world, hbm_bytes,
                              ctypes.byref(p))
    if st != KNN_OK:
        raise KnnError(st, "knn_shard_policy")
    return "train" if p.value == 1 else "test"


def exchange_layout(nq, k, world, rank):
    """knn_exchange_layout: (send_off, send_cnt, recv_off, recv_cnt) int32-element arrays of
    the train-sharded all-to-all of rank `rank`."""
    lib = load_library()
    arrs = [np.zeros(world, np.int64) for _ in range(4)]
    st = lib.knn_exchange_layout(nq, k, world, rank, *[_ptr(a) for a in arrs])
    if st != KNN_OK:
        raise KnnError(st, "knn_exchange_layout")
    return tuple(arrs)


class Comm:
    """An RCCL communicator bound to a context (knn_comm_create; collective over nranks)."""

    def __init__(self, ctx, uid, nranks, rank):
        self.lib = ctx.lib
        self.ctx = ctx
        self.nranks, self.rank = nranks, rank
        h = ctypes.c_void_p()
        st = self.lib.knn_comm_create(ctx.h, ctypes.create_string_buffer(bytes(uid), KNN_COMM_ID_BYTES), nranks,
                                      rank, ctypes.byref(h))
        if st != KNN_OK:
            raise KnnError(st, f"knn_comm_create(nranks={nranks}, rank={rank})")
        self.h = h

    def predict_train_sharded(self, shard, labels, idx_base, test, k, num_classes, pred, dist=None, idx=None,
                              stream=None, d=None):
        """knn_predict_train_sharded: this rank's train shard (global rows [idx_base, ...)) and
        every query in, the owned queries' (shard_range) predictions out."""
        self.ctx._on_device(shard)
        self.ctx._note_train(shard)
        tr = _device_dataset(shard, labels, d)
        te = _device_dataset(test, None, d)
        q0, q1 = shard_range(te.n, self.nranks, self.rank)
        _outputs(q1 - q0, k, pred, dist, idx)
        st = self.lib.knn_predict_train_sharded(
            self.ctx.h, self.h, ctypes.byref(tr), idx_base, ctypes.byref(te), k, num_classes, pred.data_ptr(),
            None if dist is None else dist.data_ptr(), None if idx is None else idx.data_ptr(),
            self.ctx._stream(stream, test))
        if st != KNN_OK:
            raise KnnError(st, self.lib.knn_last_error(self.ctx.h).decode())
        return q0, q1

    def count(self):
        """The number of ranks the RCCL communicator spans (knn_comm_count: ncclCommCount)."""
        n = ctypes.c_int32()
        st = self.lib.knn_comm_count(self.h, ctypes.byref(n))
        if st != KNN_OK:
            raise KnnError(st, "knn_comm_count")
        return n.value

    def set_exchange(self, chunk_elems=0, self_via_rccl=False):
        """knn_comm_set_exchange: RCCL messages of at most chunk_elems int32 (0: the default,
        256 MiB); self_via_rccl sends the rank's own block through the RCCL loop too (a one-rank
        communicator then runs the multi-rank exchange's offsets and counts)."""
        st = self.lib.knn_comm_set_exchange(self.h, int(chunk_elems), 1 if self_via_rccl else 0)
        if st != KNN_OK:
            raise KnnError(st, "knn_comm_set_exchange")

    def broken(self):
        """True once a collective failed and the communicator was aborted (knn_comm_broken)."""
        b = ctypes.c_int32()
        st = self.lib.knn_comm_broken(self.h, ctypes.byref(b))
        if st != KNN_OK:
            raise KnnError(st, "knn_comm_broken")
        return bool(b.value)

    def close(self):
        if getattr(self, "h", None):
            self.lib.knn_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PinnedArray:
    """A numpy array over page-locked host memory (knn_alloc_pinned / knn_free_pinned)."""

    def __init__(self, shape, dtype):
        self.lib = load_library()
        dtype = np.dtype(dtype)
        nbytes = int(np.prod(shape)) * dtype.itemsize
        p = ctypes.c_void_p()
        st = self.lib.knn_alloc_pinned(max(nbytes, 1), ctypes.byref(p))
        if st != KNN_OK:
            raise KnnError(st, f"knn_alloc_pinned({nbytes})")
        self.ptr = p
        buf = (ctypes.c_char * max(nbytes, 1)).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=dtype, count=int(np.prod(shape))).reshape(shape)

    def free(self):
        if getattr(self, "ptr", None):
            self.array = None
            self.lib.knn_free_pinned(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


_default_ctx = None


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


def read_arff(path):
    """Parse a NUMERIC ARFF file -> (features float32 [n][d], labels int32 [n], num_classes)."""
    lib = load_library()
    h = ctypes.c_void_p()
    err = ctypes.create_string_buffer(512)
    st = lib.knn_arff_open(os.fsencode(path), ctypes.byref(h), err, 512)
    if st != KNN_OK:
        raise KnnError(st, err.value.decode())
    try:
        n, na, C = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32()
        lib.knn_arff_shape(h, ctypes.byref(n), ctypes.byref(na), ctypes.byref(C))
        d = na.value - 1
        feat = np.zeros((n.value, max(d, 0)), np.float32)
        labels = np.zeros(n.value, np.int32)
        st = lib.knn_arff_copy(h, _ptr(feat), max(d, 0), _ptr(labels))
        if st != KNN_OK:
            raise KnnError(st, "non-numeric or missing value in " + str(path))
        return feat, labels, C.value
    finally:
        lib.knn_arff_close(h)


def KNN(train, test, k, ctx=None):
    """main.cpp:25 -- train = (features, labels), test = features or (features, labels).
    k <= 0 gives all-zero predictions like the reference."""
    tf, tl = train
    qf = test[0] if isinstance(test, tuple) else test
    if k <= 0:
        return np.zeros(len(qf), np.int32)
    return (ctx or default_context()).predict(tf, tl, qf, k, int(np.max(tl)) + 1)


def KNN_range(train, test, k, start, end, ctx=None):
    """mpi.cpp:26 -- predictions for test rows [start, end)."""
    tf, tl = train
    qf = test[0] if isinstance(test, tuple) else test
    if k <= 0:
        return np.zeros(end - start, np.int32)
    return (ctx or default_context()).predict(tf, tl, qf, k, int(np.max(tl)) + 1, start, end)


def computeConfusionMatrix(predictions, labels, num_classes):
    """main.cpp:87 -- [true][pred] counts, C x C int32."""
    lib = load_library()
    p = np.ascontiguousarray(predictions, np.int32)
    lab = np.ascontiguousarray(labels, np.int32)
    cm = np.zeros((num_classes, num_classes), np.int32)
    st = lib.knn_confusion_matrix(_ptr(p), _ptr(lab), len(p), num_classes, _ptr(cm))
    if st != KNN_OK:
        raise KnnError(st, "label or prediction outside [0, num_classes)")
    return cm


def computeAccuracy(cm, n):
    """main.cpp:102 -- trace / n as float32."""
    lib = load_library()
    cm = np.ascontiguousarray(cm, np.int32)
    return float(np.float32(lib.knn_accuracy(_ptr(cm), cm.shape[0], n)))
