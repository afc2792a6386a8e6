"""DataFrame / ML device ops (wrappers over csrc/kernels/df.hip and ml.hip).

GPU tensors go to the HIP kernels; CPU tensors use numpy/torch host code with the same
semantics (the ``local[N]`` executor path).  Column type codes match ``ColType`` in df.hip.
"""
from __future__ import annotations

import ctypes
import math
import os
import struct

import numpy as np
import torch

from .. import _native, config
from ._util import hip, on_device, ptr

CT_F32, CT_F64, CT_I32, CT_I64, CT_U8, CT_CODE = range(6)
TORCH_CT = {torch.float32: CT_F32, torch.float64: CT_F64, torch.int32: CT_I32, torch.int64: CT_I64,
            torch.uint8: CT_U8, torch.bool: CT_U8}

# VM opcodes (enum VmOp in df.hip)
OPS = ["", "LDCOL", "LDC", "LDNULL", "ADD", "SUB", "MUL", "DIV", "MOD", "NEG", "ABS", "SQRT", "LOG", "EXP", "POW",
       "FLOOR", "CEIL", "EQ", "NE", "LT", "LE", "GT", "GE", "AND", "OR", "NOT", "ISNULL", "ISNOTNULL", "ISNAN",
       "SELECT", "COALESCE", "CAST_INT", "EQ_NULLSAFE", "MIN2", "MAX2", "ROUND"]
OP = {n: i for i, n in enumerate(OPS) if n}
VM_INS, VM_COLS, VM_CONSTS = 96, 12, 32


def pack_ins(op: str, d: int, a: int = 0, b: int = 0, c: int = 0, k: int = 0) -> int:
    w = OP[op] | (d << 8) | (a << 12) | (b << 16) | (c << 20) | (k << 24)
    return w - (1 << 32) if w >= (1 << 31) else w


def pack_vm_prog(ins, out_reg, out_type, filter_mode, consts, cols) -> bytes:
    """cols: list of (tensor, valid_tensor_or_None, type_code)."""
    if len(ins) > VM_INS or len(consts) > VM_CONSTS or len(cols) > VM_COLS:
        raise ValueError("expression too large for the device VM")
    buf = struct.pack("4i", len(ins), out_reg, out_type, int(filter_mode))
    buf += struct.pack(f"{VM_INS}i", *(list(ins) + [0] * (VM_INS - len(ins))))
    buf += struct.pack(f"{VM_CONSTS}d", *(list(consts) + [0.0] * (VM_CONSTS - len(consts))))
    ptrs = [c[0].data_ptr() for c in cols] + [0] * (VM_COLS - len(cols))
    vptr = [(c[1].data_ptr() if c[1] is not None else 0) for c in cols] + [0] * (VM_COLS - len(cols))
    types = [c[2] for c in cols] + [0] * (VM_COLS - len(cols))
    buf += struct.pack(f"{VM_COLS}Q", *ptrs) + struct.pack(f"{VM_COLS}Q", *vptr) + struct.pack(f"{VM_COLS}i", *types)
    size = _native.hip_lib().ptg_vm_prog_size()
    buf += b"\0" * (size - len(buf))
    assert len(buf) == size, (len(buf), size)
    return buf


def expr_eval(prog: bytes, n: int, out, out_valid=None):
    cbuf = ctypes.create_string_buffer(prog, len(prog))
    hip("ptg_expr_eval", ctypes.addressof(cbuf), n, ptr(out), ptr(out_valid))


# ------------------------------------------------------------------------------------------------
# Device fills / iota (dfutil.hip): the operators use these instead of torch.zeros / ones / full /
# arange, so a DataFrame query launches only framework kernels.
def fill(t: torch.Tensor, value) -> torch.Tensor:
    """t[:] = value (contiguous t; bool / int / float of 1, 2, 4 or 8 bytes)."""
    if not on_device(t) or not t.is_contiguous():
        return t.fill_(value)
    es = t.element_size()
    if t.dtype == torch.float64:
        pat = int(np.array(value, dtype=np.float64).view(np.int64))
    elif t.dtype == torch.float32:
        pat = int(np.array(value, dtype=np.float32).view(np.int32))
    else:
        pat = int(value)
    pat &= (1 << (8 * es)) - 1
    if pat >= 1 << 63:
        pat -= 1 << 64
    hip("ptg_fill_bytes", ptr(t), t.numel(), es, pat)
    return t


def full(n: int, value, dtype, device) -> torch.Tensor:
    return fill(torch.empty(n, dtype=dtype, device=device), value)


def zeros(n: int, dtype, device) -> torch.Tensor:
    return full(n, 0, dtype, device)


def arange(start: int, stop: int, device) -> torch.Tensor:
    """int64 [start, stop)."""
    n = max(0, stop - start)
    out = torch.empty(n, dtype=torch.int64, device=device)
    if not on_device(out):
        return torch.arange(start, start + n, dtype=torch.int64)
    hip("ptg_iota_i64", ptr(out), n, int(start))
    return out


# ------------------------------------------------------------------------------------------------
def compact(mask: torch.Tensor) -> torch.Tensor:
    """Ascending int64 indices of the non-zero entries of a uint8/bool mask."""
    n = mask.numel()
    if not on_device(mask):
        return torch.nonzero(mask.view(-1).bool(), as_tuple=False).view(-1)
    m = mask.view(torch.uint8) if mask.dtype == torch.bool else mask
    nb = max(1, math.ceil(n / 4096))
    dev = mask.device
    bc = torch.empty(nb, dtype=torch.int32, device=dev)
    bo = torch.empty(nb, dtype=torch.int64, device=dev)
    tot = zeros(1, torch.int64, dev)
    hip("ptg_compact", ptr(m), n, ptr(bc), ptr(bo), ptr(tot), None)
    total = int(tot.item())
    idx = torch.empty(total, dtype=torch.int64, device=dev)
    if total:
        hip("ptg_compact", ptr(m), n, ptr(bc), ptr(bo), ptr(tot), ptr(idx))
    return idx


def gather_rows(t: torch.Tensor, idx: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """t[idx] along dim 0; ``out`` (contiguous, [idx.numel(), *t.shape[1:]]) receives the rows in place
    of a new tensor (a shuffle writes its local rows straight into their final output slice)."""
    m = idx.numel()
    if out is not None and (tuple(out.shape) != (m, *t.shape[1:]) or out.dtype != t.dtype or not out.is_contiguous()):
        raise ValueError(f"gather_rows: out {tuple(out.shape)} {out.dtype} does not fit {m} rows of {tuple(t.shape)}")
    if not on_device(t):
        return torch.index_select(t, 0, idx, out=out) if out is not None else t.index_select(0, idx)
    if out is None:
        out = torch.empty((m, *t.shape[1:]), dtype=t.dtype, device=t.device)
    if m == 0:
        return out
    row_bytes = t[0].numel() * t.element_size() if t.dim() > 0 and t.shape[0] > 0 else t.element_size()
    src = t.contiguous()
    if row_bytes in (4, 8) and idx.dtype in (torch.int64, torch.int32) and not _native.CHECKED:
        # one row per thread, 4 in flight (dfutil.hip gather_fixed_k); int32 indices are u32 row ids
        hip("ptg_gather_fixed", ptr(src), ptr(idx), int(idx.dtype == torch.int32), m, row_bytes, ptr(out))
        return out
    if idx.dtype != torch.int64:
        idx = idx.to(torch.int64)
    hip("ptg_gather_rows", ptr(src), ptr(idx), m, row_bytes, t.shape[0] if t.dim() > 0 else 1, ptr(out))
    return out


def reduce_stats(col: torch.Tensor, valid, skip_nan: bool = True):
    """-> (sum, count, min, max, nulls) as Python floats."""
    if not on_device(col):
        x = col.double()
        ok = torch.ones_like(x, dtype=torch.bool) if valid is None else valid.bool()
        if skip_nan:
            ok = ok & ~torch.isnan(x)
        v = x[ok]
        return (float(v.sum()) if v.numel() else 0.0, float(v.numel()),
                float(v.min()) if v.numel() else math.inf, float(v.max()) if v.numel() else -math.inf,
                float(x.numel() - v.numel()))
    dev = col.device
    part = torch.empty(5 * 1024, dtype=torch.float64, device=dev)
    out = torch.empty(5, dtype=torch.float64, device=dev)
    t = col if col.dtype != torch.bool else col.view(torch.uint8)
    hip("ptg_reduce_stats", ptr(t), TORCH_CT[t.dtype], ptr(valid), col.numel(), int(skip_nan), ptr(part), ptr(out))
    return tuple(float(x) for x in out.cpu().tolist())


def histogram(codes: torch.Tensor, nbins: int) -> torch.Tensor:
    """counts[nbins + 1] (int64); last bin = nulls / out-of-range."""
    if not on_device(codes):
        c = codes.long().clone()
        c[(c < 0) | (c >= nbins)] = nbins
        return torch.bincount(c, minlength=nbins + 1)
    out = torch.zeros(nbins + 1, dtype=torch.int64, device=codes.device)
    hip("ptg_histogram_i32", ptr(codes), codes.numel(), ptr(out), nbins)
    return out


# ------------------------------------------------------------------------------------------------
# small device utilities (csrc/kernels/dfutil.hip): the groupBy / sort paths launch only our kernels
# ------------------------------------------------------------------------------------------------
def scan_excl(x: torch.Tensor, out: torch.Tensor | None = None, total: torch.Tensor | None = None) -> torch.Tensor:
    """Exclusive prefix sum of an int32 / int64 vector into int64 ``out``; ``total`` (1-element
    int64 view, anywhere) receives the sum."""
    n = x.numel()
    if out is None:
        out = torch.empty(max(n, 1), dtype=torch.int64, device=x.device)[:n]
    if not on_device(x):
        cs = torch.cumsum(x.to(torch.int64), 0)
        out[:n] = cs - x.to(torch.int64)
        if total is not None:
            total.fill_(int(cs[-1]) if n else 0)
        return out
    ws = torch.empty(max(1, int(_native.hip_lib().ptg_scan_ws_elems(n))), dtype=torch.int64, device=x.device)
    hip("ptg_scan_excl", ptr(x), int(x.dtype == torch.int64), n, ptr(out), ptr(total), ptr(ws))
    return out


def minmax_i64(x: torch.Tensor, n: int | None = None, stride: int = 1, off_min: int = 0, off_max: int = 0):
    """(min over x[i*stride + off_min], max over x[i*stride + off_max]) as Python ints; ``x`` a
    contiguous int64 buffer (a strided sample of a column, or the [tiles, 2] range table)."""
    n = (x.numel() + stride - 1) // stride if n is None else n
    if not on_device(x):
        flat = x.reshape(-1)
        return int(flat[off_min::stride][:n].min()), int(flat[off_max::stride][:n].max())
    out = torch.empty(2, dtype=torch.int64, device=x.device)
    hip("ptg_minmax_i64", ptr(x), n, stride, off_min, off_max, ptr(out))
    lo, hi = out.tolist()
    return int(lo), int(hi)


def strided_sample(keys: torch.Tensor, stride: int, m: int) -> torch.Tensor:
    """keys[::stride][:m] as a contiguous int64 tensor."""
    if not on_device(keys):
        return keys[::stride][:m].contiguous()
    out = torch.empty(max(m, 1), dtype=torch.int64, device=keys.device)[:m]
    hip("ptg_strided_copy_i64", ptr(keys), stride, m, ptr(out))
    return out


def _dense_extract(prow, psum, pmm, C: int, nv: int, W: int, lo: int, dev):
    """Sum the C per-chunk partial tables of a direct-indexed aggregation and compact the occupied
    keys (dense_count_k / dense_write_k): -> (keys, rows, [(sum, cnt, min, max)] per column)."""
    nb = max(1, -(-W // 4096))
    bcount = torch.empty(nb, dtype=torch.int32, device=dev)
    boff = torch.empty(nb, dtype=torch.int64, device=dev)
    total = torch.empty(1, dtype=torch.int64, device=dev)
    if nb <= 4096:
        hip("ptg_dense_extract", ptr(prow), ptr(psum), ptr(pmm), C, nv, W, int(lo), ptr(bcount), ptr(boff),
            ptr(total), None, 1)
    else:  # windows beyond 2^24 keys (the two-level range path): block counts scanned by scan_excl
        hip("ptg_dense_extract", ptr(prow), ptr(psum), ptr(pmm), C, nv, W, int(lo), ptr(bcount), ptr(boff),
            ptr(total), None, 0)
        scan_excl(bcount, out=boff, total=total)
    m = int(total.item())
    keys = torch.empty(max(m, 1), dtype=torch.int64, device=dev)[:m]
    cols = torch.empty((1 + 4 * max(nv, 1), max(m, 1)), dtype=torch.float64, device=dev)[:, :m]
    rows = cols[0]
    outs = [(cols[1 + 4 * j], cols[2 + 4 * j], cols[3 + 4 * j], cols[4 + 4 * j]) for j in range(nv)]
    ptrs = [keys.data_ptr(), rows.data_ptr()]
    for q in range(4):  # sum, cnt, min, max
        ptrs += [outs[j][q].data_ptr() if j < nv else 0 for j in range(4)]
    arr = (ctypes.c_uint64 * 18)(*ptrs)
    if m:
        hip("ptg_dense_extract", ptr(prow), ptr(psum), ptr(pmm), C, nv, W, int(lo), ptr(bcount), ptr(boff),
            ptr(total), ctypes.addressof(arr), 2)
    return keys, rows, outs


# ------------------------------------------------------------------------------------------------
# hash aggregation
# ------------------------------------------------------------------------------------------------
def _pow2(x: int) -> int:
    return 1 << max(4, int(math.ceil(math.log2(max(x, 1)))))


def _small_range_agg(keys, vals, valids):
    """Keys spanning < ~4K values (small_range_agg_k): the whole range is one direct-indexed LDS
    table per workgroup, one pass over the rows; None when the span is wider.  The key window comes
    from a strided sample (64K loads); a key outside it makes the kernel flag an error and the pass
    is re-run on the exact range (one full min/max read of the keys, only then)."""
    n = keys.numel()
    nv = len(vals)
    keys = keys.contiguous()
    wmax = (150 * 1024) // (4 + 12 * nv)
    st = max(1, n // 65536)
    slo, shi = minmax_i64(keys, n=(n + st - 1) // st, stride=st)
    if shi - slo >= wmax:
        return None
    pay = []
    for v, vd in zip(vals, valids):
        v = v.view(torch.uint8) if v.dtype == torch.bool else v.contiguous()
        if vd is not None and vd.dtype == torch.bool:
            vd = vd.view(torch.uint8)
        pay.append((v, vd))
    fast = nv > 0 and all(v.dtype == torch.float64 and vd is None and v.data_ptr() % 16 == 0 for v, vd in pay) \
        and keys.data_ptr() % 16 == 0
    pin = _pay_in(pay)
    err = zeros(1, torch.int32, keys.device)
    # a little headroom around the sampled range: a key the sample missed just outside it still fits
    span = shi - slo + 1
    pad = min((wmax - span) // 2, span // 16 + 8)
    lo, W = slo - pad, span + 2 * pad
    G = int(config.get("groupby_small_blocks"))
    quant = 2048 if fast else 1
    rpb = -(-(-(-n // G)) // quant) * quant
    G = -(-n // rpb)
    prow = torch.empty((G, 1 + nv, W), dtype=torch.int32, device=keys.device)
    psum = torch.empty((G, max(nv, 1), W), dtype=torch.float64, device=keys.device)
    hip("ptg_small_range_agg", ptr(keys), n, lo, W, ctypes.addressof(pin), nv, rpb, G, ptr(prow),
        ptr(psum), ptr(err), int(fast))
    if int(err.item()):
        lo, hi = minmax_i64(keys)  # the sample missed keys: exact range
        W = hi - lo + 1
        if W > wmax:
            return None
        prow = torch.empty((G, 1 + nv, W), dtype=torch.int32, device=keys.device)
        psum = torch.empty((G, max(nv, 1), W), dtype=torch.float64, device=keys.device)
        fill(err, 0)
        hip("ptg_small_range_agg", ptr(keys), n, lo, W, ctypes.addressof(pin), nv, rpb, G, ptr(prow),
            ptr(psum), ptr(err), int(fast))
    if G > 64:
        # fold the per-workgroup partials 32 at a time first: the extract parallelises over keys only
        F = 32
        G2 = -(-G // F)
        prow2 = torch.empty((G2, 1 + nv, W), dtype=torch.int32, device=keys.device)
        psum2 = torch.empty((G2, max(nv, 1), W), dtype=torch.float64, device=keys.device)
        hip("ptg_dense_fold", ptr(prow), ptr(psum), G, nv, W, F, ptr(prow2), ptr(psum2))
        prow, psum, G = prow2, psum2, G2
    return _dense_extract(prow, psum, None, G, nv, W, lo, keys.device)


def hash_agg(keys: torch.Tensor, vals: list, valids: list, want_minmax: bool = False, cap_hint: int | None = None,
             est_keys: int | None = None):
    """groupBy(key).agg over int64 keys.  Returns (keys[m], rows[m], [(sum, cnt, min, max)] per value column)
    as tensors on the keys' device.  ``est_keys`` (expected distinct keys) sizes the per-workgroup LDS
    tables of hash_agg_lds_k."""
    nv = len(vals)
    n = keys.numel()
    if not on_device(keys):
        uk, inv = torch.unique(keys, return_inverse=True)
        m = uk.numel()
        rows = torch.bincount(inv, minlength=m).double()
        outs = []
        for v, vd in zip(vals, valids):
            x = v.double()
            ok = ~torch.isnan(x) if vd is None else (vd.bool() & ~torch.isnan(x))
            xs = torch.where(ok, x, torch.zeros_like(x))
            s = torch.zeros(m, dtype=torch.float64).index_add_(0, inv, xs)
            c = torch.zeros(m, dtype=torch.float64).index_add_(0, inv, ok.double())
            mn = torch.full((m,), math.inf, dtype=torch.float64).scatter_reduce_(0, inv, torch.where(ok, x, torch.full_like(x, math.inf)), "amin")
            mx = torch.full((m,), -math.inf, dtype=torch.float64).scatter_reduce_(0, inv, torch.where(ok, x, torch.full_like(x, -math.inf)), "amax")
            outs.append((s, c, mn, mx))
        return uk, rows, outs
    if (not want_minmax and keys.dtype == torch.int64 and n >= RANGE_MIN_ROWS and nv <= PAY_MAX
            and config.get("groupby_range")):
        r = _small_range_agg(keys, vals, valids)
        if r is not None:
            return r
    dev = keys.device
    cap = _pow2(2 * (cap_hint if cap_hint else min(n, 1 << 22)) + 16)
    gkeys = torch.empty(cap, dtype=torch.int64, device=dev)
    gtab = torch.empty((1 + 4 * nv) * cap, dtype=torch.float64, device=dev)
    overflow = zeros(1, torch.int32, dev)
    hip("ptg_hash_table_init", ptr(gkeys), ptr(gtab), cap, nv)
    vptrs = (ctypes.c_void_p * 4)(*[v.data_ptr() for v in vals])
    vvals = (ctypes.c_void_p * 4)(*[(vd.data_ptr() if vd is not None else 0) for vd in valids])
    types = (ctypes.c_int * 4)(*[TORCH_CT[v.dtype] for v in vals])
    hip("ptg_hash_agg", ptr(keys), n, ctypes.addressof(vptrs), ctypes.addressof(vvals), ctypes.addressof(types), nv,
        int(want_minmax), ptr(gkeys), ptr(gtab), cap, ptr(overflow), int(est_keys or cap_hint or 512))
    if int(overflow.item()):
        # table too small for the key cardinality: retry with a larger table
        return hash_agg(keys, vals, valids, want_minmax, cap_hint=cap * 2, est_keys=est_keys)
    return _extract(gkeys, gtab, cap, nv)


def _extract(gkeys, gtab, cap, nv):
    dev = gkeys.device
    mcount = zeros(1, torch.int64, dev)
    hip("ptg_hash_extract", ptr(gkeys), ptr(gtab), cap, nv, None, None, 0, ptr(mcount))
    m = int(mcount.item())
    ok = torch.empty(m, dtype=torch.int64, device=dev)
    ot = torch.empty((1 + 4 * nv) * max(m, 1), dtype=torch.float64, device=dev)
    fill(mcount, 0)
    hip("ptg_hash_extract", ptr(gkeys), ptr(gtab), cap, nv, ptr(ok), ptr(ot), m, ptr(mcount))
    ot = ot.view(1 + 4 * nv, max(m, 1))[:, :m]
    outs = [(ot[1 + 4 * j], ot[2 + 4 * j], ot[3 + 4 * j], ot[4 + 4 * j]) for j in range(nv)]
    return ok, ot[0], outs


def radix_tile(nv: int) -> int:
    """Tile rows of radix_scatter_k<nv> (RTT in df.hip: LDS holds a tile's keys + nv columns)."""
    rt = _native.hip_lib().ptg_radix_tile_rows()
    return rt if nv <= 1 else rt // 2
RADIX_BITS = 6  # digit bits per radix level (RB = 64 in df.hip)
PAY_MAX = 4  # value columns carried through a partitioning pass (PAY_MAX in df.hip)
_AGG_LDS_BUDGET = 64 * 1024  # part_agg2_k table bytes: keeps >= 2 workgroups resident per CU


def _pay_in(cols) -> ctypes.Array:
    """PayIn descriptor (df.hip) for a list of (tensor, valid u8 tensor or None)."""
    cols = list(cols)
    pad = PAY_MAX - len(cols)
    b = struct.pack(f"{PAY_MAX}Q", *([c[0].data_ptr() for c in cols] + [0] * pad))
    b += struct.pack(f"{PAY_MAX}Q", *([(c[1].data_ptr() if c[1] is not None else 0) for c in cols] + [0] * pad))
    b += struct.pack(f"{PAY_MAX}i", *([TORCH_CT[c[0].dtype] for c in cols] + [0] * pad))
    size = _native.hip_lib().ptg_pay_desc_size()
    b += b"\0" * (size - len(b))
    return ctypes.create_string_buffer(b, len(b))


def _pay_out(tensors) -> ctypes.Array:
    ts = list(tensors)
    b = struct.pack(f"{PAY_MAX}Q", *([t.data_ptr() for t in ts] + [0] * (PAY_MAX - len(ts))))
    return ctypes.create_string_buffer(b, len(b))


def _radix_level(keys, kbase, pay_cols, seg_start, seg_len, shift, buf, tag, compress=False):
    """One radix level over segments [seg_start, seg_start+seg_len) of ``keys`` (+ payload columns,
    written out as f64 with null -> NaN).  Rows are split by the 6 hash bits at ``shift``; the output
    holds the segments' rows only (n_out = sum(seg_len)), segment-major then digit-major.
    ``keys`` are int64, or int32 bit patterns of u32 offsets from ``kbase``; ``compress`` (first
    level): the count pass also finds the key range and, when max - min < 2^32 - 1, the scatter
    writes u32 offsets from min (12 instead of 16 bytes per row through every later pass).
    Returns (okeys, kbase_out, [ovals], new_start, new_end) of the nseg*64 sub-segments."""
    dev = keys.device
    T = radix_tile(len(pay_cols))
    nseg = seg_start.numel()
    # tile plan on the device (dfutil.hip): tiles per segment, their exclusive prefix, and the
    # per-tile start / rows / histogram base and stride; one readback of (tiles, rows)
    ntiles_s = buf(tag + "nts", (nseg,), torch.int64)
    hip("ptg_radix_plan", ptr(seg_start), ptr(seg_len), nseg, T, ptr(ntiles_s), None, 0, None, None, None, None, 0)
    first = buf(tag + "first", (nseg,), torch.int64)
    tot2 = buf(tag + "tot2", (2,), torch.int64)
    scan_excl(ntiles_s, out=first, total=tot2[0:1])
    lens_scan = buf(tag + "lscan", (nseg,), torch.int64)
    scan_excl(seg_len, out=lens_scan, total=tot2[1:2])
    total, n_out = (int(x) for x in tot2.tolist())
    nv = len(pay_cols)
    in32 = keys.dtype == torch.int32
    ovals = [buf(f"{tag}ov{j}", (max(n_out, 1),), torch.float64)[:n_out] for j in range(nv)]
    if total == 0:
        z = torch.zeros(nseg * 64, dtype=torch.int64, device=dev)
        return keys[:0], kbase, ovals, z, z, z
    tstart = buf(tag + "tst", (total,), torch.int64)
    trows = buf(tag + "trw", (total,), torch.int32)
    thbase = buf(tag + "thb", (total,), torch.int64)
    thstride = buf(tag + "ths", (total,), torch.int64)
    hip("ptg_radix_plan", ptr(seg_start), ptr(seg_len), nseg, T, ptr(ntiles_s), ptr(first), total, ptr(tstart),
        ptr(trows), ptr(thbase), ptr(thstride), 1)
    hist = buf(tag + "hist", (64 * total,), torch.int32)
    rng = buf(tag + "rng", (total, 2), torch.int64) if (compress and not in32) else None
    hip("ptg_radix_count", ptr(keys), int(in32), int(kbase), ptr(tstart), ptr(trows), ptr(thbase), ptr(thstride),
        total, shift, ptr(hist), ptr(rng))
    offs = buf(tag + "offs", (64 * total + 1,), torch.int64)
    scan_excl(hist, out=offs[:-1], total=offs[-1:])
    out32, kbase_out = in32, kbase
    if rng is not None:
        lo, hi = minmax_i64(rng, n=total, stride=2, off_min=0, off_max=1)
        if hi - lo < (1 << 32) - 1:
            out32, kbase_out = True, lo
    okeys = buf(tag + ("okeys32" if out32 else "okeys"), (max(n_out, 1),),
                torch.int32 if out32 else torch.int64)[:n_out]
    pin = _pay_in(pay_cols)
    pout = _pay_out(ovals)
    hip("ptg_radix_scatter", ptr(keys), int(in32), int(kbase), ctypes.addressof(pin), nv, ptr(tstart), ptr(trows),
        ptr(thbase), ptr(thstride), total, shift, ptr(offs[:-1]), n_out, ptr(okeys), int(out32), int(kbase_out),
        ctypes.addressof(pout))
    # sub-segment (s, d) starts at the run of its first tile; empty segments (no tiles) start where
    # the next non-empty one does (offs[-1] = n_out is the sentinel)
    new_start = buf(tag + "nst", (nseg * 64,), torch.int64)
    new_end = buf(tag + "nen", (nseg * 64,), torch.int64)
    new_len = buf(tag + "nln", (nseg * 64,), torch.int64)
    hip("ptg_radix_bounds", ptr(offs), ptr(first), ptr(ntiles_s), nseg, n_out, ptr(new_start), ptr(new_end),
        ptr(new_len))
    return okeys, kbase_out, ovals, new_start, new_end, new_len


def _part_agg_lds(pcap: int, nv: int, minmax: bool) -> int:
    return pcap * (8 + 4 + nv * (4 + 8 * (3 if minmax else 1)))


ESTIMATE_SAMPLE = 1 << 16
ESTIMATE_SAMPLE_MAX = 1 << 20  # the widened sample stays a few MB: never a full-size hash_agg


def estimate_distinct(keys: torch.Tensor, sample: int = ESTIMATE_SAMPLE) -> int:
    """Distinct-key estimate from a strided sample: solves d = K (1 - exp(-m/K)) for K (uniform
    key frequencies; skewed data is still handled exactly by the spill recursion)."""
    n = keys.numel()
    if n <= sample:
        return int(hash_agg(keys, [], [], False)[0].numel())
    s = strided_sample(keys.contiguous(), n // sample, sample)
    d = int(hash_agg(s, [], [], False)[0].numel())
    m = s.numel()
    if d >= 0.999 * m and n >= 16 * sample and sample * 16 <= ESTIMATE_SAMPLE_MAX:
        # a saturated sample says only "many more keys than the sample": look again 16x wider, ONCE
        # (64K -> 1M rows), before concluding every row is distinct (1B rows / 128M keys planned 4
        # radix levels and 16.7M tiny partitions from K = n: 202 ms in part_agg2_k).  Still
        # saturated at 1M rows means >~ 1e9 keys: K = n and hash_agg_radix's spill recursion copes.
        return estimate_distinct(keys, sample * 16)
    if d >= 0.999 * m:
        return n
    lo, hi = float(d), float(n)
    for _ in range(60):
        mid = math.sqrt(lo * hi)
        if mid * (1.0 - math.exp(-m / mid)) < d:
            lo = mid
        else:
            hi = mid
    return int(min(n, max(d, hi)))


RANGE_MAX_SPAN = 1 << 20  # dense-key path: keys within 256 partitions x <= 4096 keys (fewer with more columns)
RANGE_MIN_ROWS = 1 << 22  # below this the sample/plan overhead is not worth a second code path


def _range_sh_max(nv: int, minmax: bool) -> int:
    """Widest partition window (log2, <= 12 = 4096 keys) whose direct-indexed LDS table fits range_agg_k's
    150 KB: 4 B of row count + per column 12 B (sum, count) and 16 B more with min/max per key."""
    per = 4 + nv * (12 + (16 if minmax else 0))
    sh = 12
    while sh > 0 and (per << sh) > 150 * 1024:
        sh -= 1
    return sh


def _range_window(lo: int, hi: int, sh_max: int = 12):
    """(window base, sh): a window of 256 << sh >= hi - lo + 1 keys (sh <= sh_max) centred on [lo, hi],
    so keys a sample missed just past its ends still fall inside; None if the span is too wide."""
    span = hi - lo + 1
    sh = 0
    while (RADIX_RANGE_BINS << sh) < span:
        sh += 1
    return None if sh > sh_max else (lo - ((RADIX_RANGE_BINS << sh) - span) // 2, sh)


RADIX_RANGE_BINS = 256


def hash_agg_range(keys: torch.Tensor, pay: list, buf, nv: int, sample_lohi: tuple[int, int],
                   minmax: bool = False):
    """groupBy(key).agg for int64 keys spanning at most 2^20 values (csrc/kernels/df.hip range_*_k):
    one range-partitioning pass by the top 8 bits of (key - lo) and a direct-indexed LDS aggregation
    per (partition, chunk), instead of the two hash levels of :func:`hash_agg_radix`.  ``sample_lohi``
    guesses the window from a sample; the count pass returns the exact [min, max] and a key outside
    the guess re-plans the window (or returns None: the caller takes the hash path).  Same result
    format as :func:`hash_agg` (min/max are +-inf unless ``minmax``)."""
    dev = keys.device
    n = keys.numel()
    lib = _native.hip_lib()
    T = int(lib.ptg_range_tile_rows(nv))
    ntiles = (n + T - 1) // T
    sh_max = _range_sh_max(nv, minmax)
    win = _range_window(*sample_lohi, sh_max)
    if win is None:
        return None
    hist = buf("rhist", (256 * ntiles,), torch.int32)
    rng = buf("rrng", (ntiles, 2), torch.int64)
    for attempt in range(2):
        lo, sh = win
        hip("ptg_range_count", ptr(keys), n, int(lo), sh, T, ntiles, ptr(hist), ptr(rng))
        mn, mx = minmax_i64(rng, n=ntiles, stride=2, off_min=0, off_max=1)
        if mn >= lo and mx < lo + (256 << sh):
            break
        win = _range_window(mn, mx, sh_max) if attempt == 0 else None
        if win is None:
            return None
    offs = buf("roffs", (256 * ntiles + 1,), torch.int64)
    digit_offsets(hist, ntiles, offs, buf)
    okeys = buf("rokeys16", (max(n, 1),), torch.int16)[:n]  # u16 index inside the partition's window
    ovals = [buf(f"aov{j}", (max(n, 1),), torch.float64)[:n] for j in range(nv)]
    pin, pout = _pay_in(pay), _pay_out(ovals)
    hip("ptg_range_scatter", ptr(keys), ctypes.addressof(pin), nv, n, int(lo), sh, ntiles, ptr(offs), ptr(okeys),
        ctypes.addressof(pout))
    Rw = 256 << sh
    chunks = max(1, min(int(config.get("groupby_range_chunks")), (n // 256) // (1 << 16) or 1))
    prow = buf("rprow", (chunks, 1 + nv, Rw), torch.int32)
    psum = buf("rpsum", (chunks, max(nv, 1), Rw), torch.float64)
    pmm = buf("rpmm", (chunks, 2 * max(nv, 1), Rw), torch.float64) if minmax else None
    vptrs = (ctypes.c_void_p * PAY_MAX)(*([o.data_ptr() for o in ovals] + [0] * (PAY_MAX - nv)))
    hip("ptg_range_agg", ptr(okeys), ctypes.addressof(vptrs), nv, int(minmax), ptr(offs), ntiles, sh, chunks,
        ptr(prow), ptr(psum), ptr(pmm) if minmax else None)
    return _dense_extract(prow, psum, pmm if minmax else None, chunks, nv, Rw, lo, dev)


RANGE2_MAX_SPAN = 1 << 28  # two 256-way range levels x 4096-key LDS windows


def hash_agg_range2(keys: torch.Tensor, pay: list, buf, nv: int, sample_lohi: tuple[int, int]):
    """groupBy(key).agg (sum / count / avg, nv <= 2, no min/max) for int64 keys spanning 2^20 .. 2^28
    values (csrc/kernels/df.hip range2_*): a coarse 256-way range pass (u32 window offsets), a fine
    256-way pass inside every coarse partition (u16 offsets) and a direct-indexed LDS aggregation per
    fine partition - two partitioning passes and no hashing, where the hash path needs three radix
    levels and LDS hash tables.  None when the keys do not fit (the caller falls back)."""
    if nv > 2:
        return None
    dev = keys.device
    n = keys.numel()
    lib = _native.hip_lib()
    sh2_max = min(12, _range_sh_max(nv, False))
    win = _range_window(*sample_lohi, sh2_max + 8)
    if win is None or win[1] < 8:
        return None
    T = int(lib.ptg_range_tile_rows(nv))
    ntiles = (n + T - 1) // T
    hist = buf("rhist", (256 * ntiles,), torch.int32)
    rng = buf("rrng", (ntiles, 2), torch.int64)
    for attempt in range(2):
        lo, sh1 = win
        hip("ptg_range_count", ptr(keys), n, int(lo), sh1, T, ntiles, ptr(hist), ptr(rng))
        mn, mx = minmax_i64(rng, n=ntiles, stride=2, off_min=0, off_max=1)
        if mn >= lo and mx < lo + (256 << sh1):
            break
        win = _range_window(mn, mx, sh2_max + 8) if attempt == 0 else None
        if win is None or win[1] < 8:
            return None
    sh2 = sh1 - 8
    offs = buf("roffs", (256 * ntiles + 1,), torch.int64)
    digit_offsets(hist, ntiles, offs, buf)
    ok32 = buf("r2ok32", (max(n, 1),), torch.int32)[:n]
    ov1 = [buf(f"r2ov1_{j}", (max(n, 1),), torch.float64)[:n] for j in range(nv)]
    pin, pout = _pay_in(pay), _pay_out(ov1)
    hip("ptg_range_scatter32", ptr(keys), ctypes.addressof(pin), nv, n, int(lo), sh1, ntiles, ptr(offs), ptr(ok32),
        ctypes.addressof(pout))
    # coarse partition c = rows [offs[c], offs[c+1]) (tile 0's row of the tile-major offsets)
    seg_start = offs[:256]
    bounds = torch.cat([offs[:256], offs[256 * ntiles:256 * ntiles + 1]])
    seg_len = bounds[1:] - bounds[:-1]
    nts = buf("r2nts", (256,), torch.int64)
    hip("ptg_seg_plan", ptr(seg_start), ptr(seg_len), 256, T, ptr(nts), None, 0, None, None, None, None, 0, 256)
    first = buf("r2first", (256,), torch.int64)
    tot = buf("r2tot", (1,), torch.int64)
    scan_excl(nts, out=first, total=tot)
    total = int(tot.item())
    tstart = buf("r2tst", (total,), torch.int64)
    trows = buf("r2trw", (total,), torch.int32)
    thbase = buf("r2thb", (total,), torch.int64)
    thstride = buf("r2ths", (total,), torch.int64)
    hip("ptg_seg_plan", ptr(seg_start), ptr(seg_len), 256, T, ptr(nts), ptr(first), total, ptr(tstart), ptr(trows),
        ptr(thbase), ptr(thstride), 1, 256)
    hist2 = buf("r2hist", (256 * total,), torch.int32)
    hip("ptg_range2_count", ptr(ok32), ptr(tstart), ptr(trows), ptr(thbase), ptr(thstride), total, nv, sh2,
        ptr(hist2))
    offs2 = buf("r2offs", (256 * total + 1,), torch.int64)
    scan_excl(hist2, out=offs2[:-1], total=offs2[-1:])
    ok16 = buf("rokeys16", (max(n, 1),), torch.int16)[:n]
    ov2 = [buf(f"aov{j}", (max(n, 1),), torch.float64)[:n] for j in range(nv)]
    vin = (ctypes.c_void_p * PAY_MAX)(*([o.data_ptr() for o in ov1] + [0] * (PAY_MAX - nv)))
    pout2 = _pay_out(ov2)
    hip("ptg_range2_scatter", ptr(ok32), ctypes.addressof(vin), nv, ptr(tstart), ptr(trows), ptr(thbase),
        ptr(thstride), total, sh2, ptr(offs2), n, ptr(ok16), ctypes.addressof(pout2))
    nfine = 256 * 256
    fstart = buf("r2fst", (nfine,), torch.int64)
    fend = buf("r2fen", (nfine,), torch.int64)
    flen = buf("r2fln", (nfine,), torch.int64)
    hip("ptg_seg_bounds", ptr(offs2), ptr(first), ptr(nts), 256, n, ptr(fstart), ptr(fend), ptr(flen), 256)
    Rw = nfine << sh2
    chunks = 1
    prow = buf("r2prow", (chunks, 1 + nv, Rw), torch.int32)
    psum = buf("r2psum", (chunks, max(nv, 1), Rw), torch.float64)
    vptrs = (ctypes.c_void_p * PAY_MAX)(*([o.data_ptr() for o in ov2] + [0] * (PAY_MAX - nv)))
    hip("ptg_range2_agg", ptr(ok16), ctypes.addressof(vptrs), nv, ptr(fstart), ptr(fend), nfine, chunks, sh2,
        ptr(prow), ptr(psum))
    return _dense_extract(prow, psum, None, chunks, nv, Rw, lo, dev)


H9_BINS = 512
# the recursive path runs two 64-way levels for any >= 1M-row input (partition parallelism), so one
# 512-way hash9 pass wins from the smallest cardinality the LDS-table path hands over (4096 keys,
# sql/dataframe.py _RADIX_MIN_KEYS): 4K sparse keys over 1B rows took 82.7 ms on the two levels
H9_MIN_KEYS = 1 << 12


def _h9_table_slots(est_keys: int, nv: int) -> int | None:
    """LDS hash-table slots per partition of hash9_agg_k / hash9_merge_k: a power of two >= 1024
    holding the expected keys of the fullest of the 512 partitions (mean + ~7%) at load <= 0.7, within
    the 150 KB LDS budget (12 + 12 nv bytes per slot); None when no such table fits."""
    need = est_keys / H9_BINS * 1.15 / 0.7
    ts = 1024
    while ts < need:
        ts *= 2
    return ts if ts * (12 + 12 * nv) <= 150 * 1024 else None


def hash_agg_h9(keys: torch.Tensor, pay: list, buf, nv: int, est_keys: int):
    """groupBy(key).agg (sum / count / avg, nv <= 2 columns) for int64 keys of mid cardinality
    (~64K..1.3M groups) in ONE partitioning pass (csrc/kernels/df.hip hash9_*_k): 512 partitions by the
    top 9 bits of mix64(key), each aggregated into an LDS hash table by chunks and the chunks folded by
    a per-partition merge.  Same result format as :func:`hash_agg` (min / max are +-inf).  Returns None
    when a table overflowed (estimate far too low): the caller then takes :func:`hash_agg_radix`'s
    recursive levels."""
    ts = _h9_table_slots(est_keys, nv)
    if ts is None or nv > 2:
        return None
    dev = keys.device
    n = keys.numel()
    lib = _native.hip_lib()
    T = int(lib.ptg_hash9_tile_rows(nv))
    ntiles = (n + T - 1) // T
    hist = buf("h9hist", (H9_BINS * ntiles,), torch.int32)
    hip("ptg_hash9_count", ptr(keys), n, T, ntiles, ptr(hist))
    offs = buf("h9offs", (H9_BINS * ntiles + 1,), torch.int64)
    tpc = DIGIT_OFFS_TPC
    nch = -(-ntiles // tpc)
    csum = buf("h9_csum", (H9_BINS * nch,), torch.int64)
    cbase = buf("h9_cbase", (H9_BINS * nch,), torch.int64)
    hip("ptg_digit_offsets_b", 0, ptr(hist), ntiles, tpc, ptr(csum), nch, None, H9_BINS, 0)
    scan_excl(csum, out=cbase, total=offs[H9_BINS * ntiles:])
    hip("ptg_digit_offsets_b", 1, ptr(hist), ntiles, tpc, ptr(cbase), nch, ptr(offs), H9_BINS, 0)
    okeys = buf("h9okeys", (max(n, 1),), torch.int64)[:n]
    ovals = [buf(f"h9ov{j}", (max(n, 1),), torch.float64)[:n] for j in range(nv)]
    pin, pout = _pay_in(pay), _pay_out(ovals)
    hip("ptg_hash9_scatter", ptr(keys), ctypes.addressof(pin), nv, n, ntiles, ptr(offs), ptr(okeys),
        ctypes.addressof(pout))
    C = max(1, int(config.get("groupby_h9_chunks")))
    R = H9_BINS * C * ts
    pkeys = buf("h9pk", (R,), torch.int64)
    prow = buf("h9pr", (R,), torch.int32)
    psum = buf("h9ps", (max(nv, 1) * R,), torch.float64)
    pcnt = buf("h9pc", (max(nv, 1) * R,), torch.int32)
    pn = buf("h9pn", (H9_BINS * C,), torch.int32)
    state = buf("h9st", (2,), torch.int64)
    vptrs = (ctypes.c_void_p * PAY_MAX)(*([o.data_ptr() for o in ovals] + [0] * (PAY_MAX - nv)))
    hip("ptg_hash9_agg", ptr(okeys), ctypes.addressof(vptrs), nv, ptr(offs), ntiles, ts, C, ptr(pkeys), ptr(prow),
        ptr(psum), ptr(pcnt), ptr(pn), ptr(state))
    cap = H9_BINS * ts
    out_keys = torch.empty(cap, dtype=torch.int64, device=dev)
    out_tab = torch.empty((1 + 4 * nv) * cap, dtype=torch.float64, device=dev)
    hip("ptg_hash9_merge", ptr(pkeys), ptr(prow), ptr(psum), ptr(pcnt), ptr(pn), nv, ts, C, ptr(out_keys),
        ptr(out_tab), cap, ptr(state))
    m, err = (int(x) for x in state.tolist())
    if err:
        return None
    ot = out_tab.view(1 + 4 * nv, cap)[:, :m]
    outs = [(ot[1 + 4 * j], ot[2 + 4 * j], ot[3 + 4 * j], ot[4 + 4 * j]) for j in range(nv)]
    return out_keys[:m], ot[0], outs


def hash_agg_radix(keys: torch.Tensor, vals: list, valids: list, want_minmax: bool = False, ws: dict | None = None,
                   est_keys: int | None = None):
    """groupBy(key).agg over int64 keys by recursive radix partitioning (high cardinality, any
    number of distinct keys).  Same result format as :func:`hash_agg`: (keys[m], rows[m],
    [(sum, cnt, min, max)] per value column); at most PAY_MAX value columns per call."""
    nv = len(vals)
    if nv > PAY_MAX:
        raise ValueError(f"hash_agg_radix: at most {PAY_MAX} value columns per call")
    if not on_device(keys):
        return hash_agg(keys, vals, valids, want_minmax)
    dev = keys.device
    n = keys.numel()
    ws = ws if ws is not None else {}

    def buf(name, shape, dtype):
        t = ws.get(name)
        numel = int(np.prod(shape))
        if t is None or t.numel() < numel or t.dtype != dtype:
            ws.pop(name, None)
            t = torch.empty(numel, dtype=dtype, device=dev)
            ws[name] = t
        return t[:numel].view(shape)

    pay = []
    for v, vd in zip(vals, valids):
        v = v.view(torch.uint8) if v.dtype == torch.bool else v
        if vd is not None and vd.dtype == torch.bool:
            vd = vd.view(torch.uint8)
        pay.append((v.contiguous(), vd))
    if keys.dtype == torch.int64 and n >= RANGE_MIN_ROWS and config.get("groupby_range"):
        st_ = max(1, n // 65536)
        slo, shi = minmax_i64(keys.contiguous(), n=(n + st_ - 1) // st_, stride=st_)
        if shi - slo < (RADIX_RANGE_BINS << _range_sh_max(nv, want_minmax)):
            r = hash_agg_range(keys.contiguous(), pay, buf, nv, (slo, shi), want_minmax)
            if r is not None:
                return r
        elif (not want_minmax and nv <= 2 and shi - slo < RANGE2_MAX_SPAN // 2 and config.get("groupby_range2")
              and (shi - slo) < 4 * n):
            # a dense wide span (a sample covering it densely: at least ~1 row per 4 keys)
            r = hash_agg_range2(keys.contiguous(), pay, buf, nv, (slo, shi))
            if r is not None:
                return r
    K = est_keys if est_keys is not None else estimate_distinct(keys)
    if (keys.dtype == torch.int64 and n >= RANGE_MIN_ROWS and nv <= 2 and not want_minmax and K >= H9_MIN_KEYS
            and config.get("groupby_hash9")):
        r = hash_agg_h9(keys.contiguous(), pay, buf, nv, K)
        if r is not None:
            return r
    pcap_max = 256
    while _part_agg_lds(pcap_max * 2, nv, want_minmax) <= _AGG_LDS_BUDGET and pcap_max < 4096:
        pcap_max *= 2
    levels = 1 if n < (1 << 20) else 2
    while K / (64 ** levels) > pcap_max / 2 and levels < 4:
        levels += 1
    P = 64 ** levels
    pcap = 256
    while pcap < pcap_max and pcap < 4 * K / P:
        pcap *= 2
    seg_start = torch.tensor([0], dtype=torch.int64).to(dev)  # host -> device copies, no fill kernels
    seg_len = torch.tensor([n], dtype=torch.int64).to(dev)
    cur_keys, cur_pay, kbase = keys.contiguous(), pay, 0
    shift = 64 - RADIX_BITS
    tags = ["a", "b"]
    lvl = 0
    pend = None
    for _ in range(levels):
        cur_keys, kbase, ov, seg_start, pend, seg_len = _radix_level(cur_keys, kbase, cur_pay, seg_start, seg_len,
                                                                     shift, buf, tags[lvl % 2], compress=(lvl == 0))
        cur_pay = [(o, None) for o in ov]
        shift -= RADIX_BITS
        lvl += 1
    res_k, res_t = [], []
    capbuf = torch.empty(1, dtype=torch.int64, device=dev)
    while True:
        P = seg_start.numel()
        hip("ptg_sum_clamp_i64", ptr(seg_len), P, pcap, ptr(capbuf))
        cap = int(capbuf.item())
        out_keys = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        out_tab = torch.empty((1 + 4 * nv) * max(cap, 1), dtype=torch.float64, device=dev)
        m_out = torch.empty(1, dtype=torch.int64, device=dev)  # zeroed by ptg_part_agg2
        spilled = torch.empty(P, dtype=torch.int32, device=dev)
        nspill = torch.empty(1, dtype=torch.int32, device=dev)
        vptrs = (ctypes.c_void_p * PAY_MAX)(*([c[0].data_ptr() for c in cur_pay] + [0] * (PAY_MAX - nv)))
        hip("ptg_part_agg2", ptr(cur_keys), int(cur_keys.dtype == torch.int32), int(kbase), ctypes.addressof(vptrs), nv,
            int(want_minmax), ptr(seg_start), ptr(pend), P, pcap, ptr(out_keys), ptr(out_tab), max(cap, 1), ptr(m_out),
            ptr(spilled), ptr(nspill))
        m = int(m_out.item())
        if m > cap:
            raise RuntimeError(f"hash_agg_radix: {m} groups exceed the output capacity {cap}")
        res_k.append(out_keys[:m])
        res_t.append(out_tab.view(1 + 4 * nv, max(cap, 1))[:, :m])
        ns = int(nspill.item())
        if ns == 0:
            break
        if shift < 16:
            raise RuntimeError("hash_agg_radix: partition recursion did not converge")
        sp = spilled[:ns].long()
        # re-partition only the spilled partitions, one level deeper
        cur_keys, kbase, ov, seg_start, pend, seg_len = _radix_level(
            cur_keys, kbase, cur_pay, seg_start[sp].contiguous(), seg_len[sp].contiguous(), shift, buf, tags[lvl % 2])
        cur_pay = [(o, None) for o in ov]
        shift -= RADIX_BITS
        lvl += 1
    ok = res_k[0] if len(res_k) == 1 else torch.cat(res_k)
    ot = res_t[0] if len(res_t) == 1 else torch.cat(res_t, dim=1)
    outs = [(ot[1 + 4 * j], ot[2 + 4 * j], ot[3 + 4 * j], ot[4 + 4 * j]) for j in range(nv)]
    return ok, ot[0], outs


def partition_perm(part: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """Row indices grouped by destination partition (stable within a block of rows)."""
    n = part.numel()
    P = counts.numel()
    if not on_device(part):
        return torch.from_numpy(np.argsort(part.numpy(), kind="stable").astype(np.int64))
    cursor = scan_excl(counts.contiguous())
    perm = torch.empty(n, dtype=torch.int64, device=part.device)
    hip("ptg_partition_perm", ptr(part), n, P, ptr(cursor), ptr(perm))
    return perm


def hash_partition(keys: torch.Tensor, P: int):
    """-> (perm[n] int64 rows grouped by destination partition, counts[P] int64)."""
    n = keys.numel()
    if not on_device(keys):
        k = keys.numpy().astype(np.uint64)
        h = _mix64_np(k) % np.uint64(P)
        perm = np.argsort(h, kind="stable")
        counts = np.bincount(h.astype(np.int64), minlength=P)
        return torch.from_numpy(perm.astype(np.int64)), torch.from_numpy(counts.astype(np.int64))
    dev = keys.device
    part = torch.empty(n, dtype=torch.int32, device=dev)
    counts = zeros(P, torch.int64, dev)
    hip("ptg_hash_partition", ptr(keys), n, P, ptr(part), ptr(counts))
    return partition_perm(part, counts), counts


# ------------------------------------------------------------------------------------------------
# sort (stable LSD radix over unsigned-orderable 64-bit keys)
# ------------------------------------------------------------------------------------------------
_U64 = (1 << 64) - 1
_SIGN = np.uint64(1 << 63)


def _signed(u: int) -> int:
    return u - (1 << 64) if u >= (1 << 63) else u


def _orderable_np(x: torch.Tensor, desc: bool) -> np.ndarray:
    a = x.numpy()
    if a.dtype.kind == "f":
        f = a.astype(np.float64)
        f = np.where(np.isnan(f), np.nan, f) + 0.0  # canonical NaN (sorts above +inf), -0 -> +0
        b = f.view(np.uint64)
        u = np.where((b >> np.uint64(63)) != 0, ~b, b | _SIGN)
    elif a.dtype in (np.uint8, np.bool_):
        u = a.astype(np.uint64)
    else:
        u = a.astype(np.int64).view(np.uint64) ^ _SIGN
    return ~u if desc else u


def sort_key(col: torch.Tensor, desc: bool = False, write: bool = True):
    """Column -> (int64 tensor holding unsigned-orderable u64 keys, lo, hi) with lo/hi the key range
    as Python ints in [0, 2^64).  ``write=False`` (device): the range only, keys None (an int64
    column then goes into :func:`radix_sort_u64` raw, with ``xin = orderable_mask(desc)``)."""
    n = col.numel()
    if not on_device(col):
        u = _orderable_np(col.contiguous(), desc)
        lo, hi = (int(u.min()), int(u.max())) if n else (0, 0)
        return torch.from_numpy(u.view(np.int64).copy()), lo, hi
    c = col.view(torch.uint8) if col.dtype == torch.bool else col.contiguous()
    out = torch.empty(n, dtype=torch.int64, device=col.device) if write else None
    rng = torch.tensor([-1, 0], dtype=torch.int64, device=col.device)
    if n:
        hip("ptg_sort_key_prep", ptr(c), TORCH_CT[c.dtype], n, int(desc), ptr(out), ptr(rng))
    lo, hi = (x & _U64 for x in rng.cpu().tolist())
    return out, (lo if n else 0), (hi if n else 0)


def sort_range_count(keys: torch.Tensor, xin: int):
    """(lo, hi, hist0) of the orderable keys ``keys ^ xin`` in one read (device int64 column): the key
    range and every sort tile's 256-bin histogram of the raw low byte, which
    :func:`radix_sort_u64` (``hist0=``) uses as its first pass's counts."""
    n = keys.numel()
    ntiles = -(-n // _native.hip_lib().ptg_sort_tile_rows())
    hist = torch.empty(256 * ntiles, dtype=torch.int32, device=keys.device)
    tmm = torch.empty(2 * ntiles, dtype=torch.int64, device=keys.device)
    rng = torch.tensor([-1, 0], dtype=torch.int64, device=keys.device)
    hip("ptg_sort_range_count", ptr(keys), n, xin, ptr(hist), ptr(tmm), ptr(rng))
    lo, hi = (x & _U64 for x in rng.cpu().tolist())
    return lo, hi, hist


def orderable_mask(desc: bool) -> int:
    """XOR mask taking an int64 value to its unsigned-orderable key (and back): the sign bit for
    ascending order, its complement for descending (as a signed int64)."""
    return _signed((1 << 63) if not desc else (1 << 63) - 1)


def decode_sort_key(sk: torch.Tensor, dtype, desc: bool) -> torch.Tensor:
    """Inverse of :func:`sort_key` for integer columns: orderable u64 bit patterns -> values."""
    if on_device(sk) and dtype in (torch.int64, torch.int32) and sk.is_contiguous():
        out = torch.empty(sk.numel(), dtype=dtype, device=sk.device)
        hip("ptg_sort_key_decode", ptr(sk), sk.numel(), int(desc), int(dtype == torch.int32), ptr(out))
        return out
    u = ~sk if desc else sk
    x = u ^ torch.iinfo(torch.int64).min  # flip the sign bit back
    return x if dtype == torch.int64 else x.to(dtype)


DIGIT_OFFS_TPC = 64  # tiles per column-scan chunk (ptg_digit_offsets)


def digit_offsets(hist: torch.Tensor, ntiles: int, offs: torch.Tensor, buf, rot: int = 0) -> torch.Tensor:
    """offs[t*256 + d] (int64, tile-major) = the stable output position of tile t's digit-d run, i.e.
    the digit-major exclusive scan of the tile-major [ntiles][256] counts ``hist``; offs[256*ntiles]
    = total.  ``buf(name, shape, dtype)`` supplies workspace.  ``rot``: digit d's counts are in column
    (d + rot) % 256 of ``hist``."""
    tpc = DIGIT_OFFS_TPC
    nch = -(-ntiles // tpc)
    csum = buf("do_csum", (256 * nch,), torch.int64)
    cbase = buf("do_cbase", (256 * nch,), torch.int64)
    hip("ptg_digit_offsets", 0, ptr(hist), ntiles, tpc, ptr(csum), nch, None, rot)
    scan_excl(csum, out=cbase, total=offs[256 * ntiles: 256 * ntiles + 1])
    hip("ptg_digit_offsets", 1, ptr(hist), ntiles, tpc, ptr(cbase), nch, ptr(offs), rot)
    return offs


def radix_sort_u64(keys: torch.Tensor, vals: torch.Tensor | None = None, lo: int = 0, hi: int = _U64,
                   row_payload: bool = False, xin: int = 0, xout: int = 0, hist0: torch.Tensor | None = None):
    """Stable sort of u64 keys (held in an int64 tensor) with an int64 payload (default: the row
    index, i.e. the result payload is the sorting permutation).  Only the significant bits of
    hi - lo are sorted: ceil(bits / 8) LSD passes of sort_count_k + sort_scatter_k.
    ``row_payload``: ``vals`` holds row ids < 2^32 (a permutation), so it may travel as u32.
    ``xin`` / ``xout``: XOR masks the first pass applies to the keys as read and the last pass as
    written (:func:`orderable_mask`: raw int64 column in, decoded column values out - no separate
    key prep / decode passes); with no pass at all (one distinct key) they must be equal.
    ``hist0``: the first pass's per-tile raw low-byte counts from :func:`sort_range_count` (no
    first count pass)."""
    n = keys.numel()
    if not on_device(keys):
        k = keys ^ xin if xin else keys
        u = k.numpy().view(np.uint64)
        order = np.argsort(u, kind="stable")
        v = torch.from_numpy(order.astype(np.int64)) if vals is None else vals[torch.from_numpy(order)]
        ko = k[torch.from_numpy(order)]
        return (ko ^ xout if xout else ko), v
    dev = keys.device
    bits = (hi - lo).bit_length()
    passes = (bits + 7) // 8
    if n == 0 or passes == 0:
        if xin != xout:
            keys = keys ^ (xin ^ xout)
        return keys, (torch.arange(n, dtype=torch.int64, device=dev) if vals is None else vals)
    ntiles = -(-n // _native.hip_lib().ptg_sort_tile_rows())
    hist = hist0 if hist0 is not None else torch.empty(256 * ntiles, dtype=torch.int32, device=dev)
    offs = torch.empty(256 * ntiles + 1, dtype=torch.int64, device=dev)
    dws: dict = {}

    def dbuf(name, shape, dtype):
        t = dws.get(name)
        if t is None:
            t = dws[name] = torch.empty(int(np.prod(shape)), dtype=dtype, device=dev)
        return t.view(shape)
    # row-index payloads travel as u32 when the rows fit 32 bits (12 instead of 16 B per row per pass)
    v32 = n <= (1 << 32) and (vals is None or row_payload)
    vdt = torch.int32 if v32 else torch.int64
    ka = keys.contiguous()
    va = None if vals is None else (vals.to(torch.int32) if v32 else vals.contiguous())
    kb = torch.empty(n, dtype=torch.int64, device=dev)
    vb = torch.empty(n, dtype=vdt, device=dev)
    kc = vc = None
    base = _signed(lo)
    for p in range(passes):
        shift = 8 * p
        pin = xin if p == 0 else 0
        pout = xout if p == passes - 1 else 0
        if p == 0 and hist0 is not None:
            digit_offsets(hist, ntiles, offs, dbuf, rot=lo & 255)
        else:
            hip("ptg_sort_count", ptr(ka), n, base, shift, ptr(hist), pin)
            digit_offsets(hist, ntiles, offs, dbuf)
        hip("ptg_sort_scatter", ptr(ka), ptr(va), n, base, shift, ptr(offs), ptr(kb), ptr(vb), int(v32), pin, pout)
        if kc is None:  # third buffer pair so the caller's keys/vals are never overwritten
            kc = torch.empty(n, dtype=torch.int64, device=dev)
            vc = torch.empty(n, dtype=vdt, device=dev)
            ka, va, kb, vb = kb, vb, kc, vc
        else:
            ka, va, kb, vb = kb, vb, ka, va
    if v32:  # u32 row ids (n may reach 2^32) widened to int64 in one pass
        hip("ptg_widen_u32", ptr(va), n, ptr(kb))  # kb: our spare int64 buffer (never the caller's keys)
        va = kb
    return ka, va


def argsort_columns(cols) -> torch.Tensor | None:
    """Stable multi-column argsort (Spark orderBy): ``cols`` = [(data, null mask or None, desc)] in
    priority order; nulls first for ascending, last for descending (Spark's defaults).  LSD over
    columns: the lowest-priority column is sorted first and every later pass is stable."""
    perm = None
    for data, null, desc in reversed(list(cols)):
        src = data if perm is None else gather_rows(data, perm)
        k, lo, hi = sort_key(src, desc)
        _, perm = radix_sort_u64(k, perm, lo, hi, row_payload=True)
        if null is not None:
            nl = gather_rows(null.to(torch.uint8).contiguous(), perm)
            flag = nl.long() if desc else (1 - nl.long())  # key 0 sorts first
            _, perm = radix_sort_u64(flag, perm, 0, 1, row_payload=True)
    return perm


def range_partition(keys: torch.Tensor, splitters: torch.Tensor, P: int):
    """-> (part int32[n], counts int64[P]): destination = number of splitters below the key
    (unsigned order; equal keys always land together)."""
    n = keys.numel()
    ns = splitters.numel()
    if not on_device(keys):
        u = keys.numpy().view(np.uint64)
        sp = splitters.numpy().view(np.uint64)
        part = np.searchsorted(sp, u, side="left").astype(np.int32)
        return torch.from_numpy(part), torch.from_numpy(np.bincount(part, minlength=P).astype(np.int64))
    part = torch.empty(n, dtype=torch.int32, device=keys.device)
    counts = zeros(P, torch.int64, keys.device)
    sp = splitters.to(keys.device).contiguous()
    hip("ptg_range_partition", ptr(keys), n, ptr(sp), ns, ptr(part), ptr(counts))
    return part, counts


def _mix64_np(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x.copy()
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xff51afd7ed558ccd)
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xc4ceb9fe1a85ec53)
        x ^= x >> np.uint64(33)
    return x


def fill_synthetic_kv(n: int, num_keys: int, device, offset: int = 0, seed: int = 42, sparse: bool = False):
    """(key, value) rows: key = hash(row) % num_keys (``sparse``: that dense key mixed over the whole
    int64 range, same number of distinct keys), value uniform in [0, 1)."""
    keys = torch.empty(n, dtype=torch.int64, device=device)
    vals = torch.empty(n, dtype=torch.float64, device=device)
    if torch.device(device).type != "cuda":
        i = np.arange(offset, offset + n, dtype=np.uint64)
        with np.errstate(over="ignore"):
            h = _mix64_np(i * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed))
            k = h % np.uint64(num_keys)
            if sparse:
                k = _mix64_np(k + np.uint64(1))
            keys.copy_(torch.from_numpy(k.view(np.int64) if sparse else k.astype(np.int64)))
            v = (_mix64_np(h ^ np.uint64(0x632BE59BD9B4E019)) >> np.uint64(11)).astype(np.float64) / 9007199254740992.0
        vals.copy_(torch.from_numpy(v))
        return keys, vals
    hip("ptg_fill_synthetic_kv", ptr(keys), ptr(vals), n, offset, num_keys, seed, int(sparse))
    return keys, vals


# ------------------------------------------------------------------------------------------------
# ML kernels
# ------------------------------------------------------------------------------------------------
def assemble_features(segments, n: int, D: int, device):
    """segments: list of (kind, tensor, offset, V, R) with kind 'onehot' (int32 codes), 'f64', 'f32'."""
    out = torch.empty((n, D), dtype=torch.float32, device=device)
    if torch.device(device).type != "cuda":
        out.zero_()
        for kind, t, off, V, R in segments:
            if kind == "onehot":
                c = t.long()
                ok = (c >= 0) & (c < V)
                rows = torch.nonzero(ok).view(-1)
                for r in range(R):
                    out[rows, off + r * V + c[rows]] = 1.0
            else:
                out[:, off] = t.float()
        return out
    kinds = {"onehot": 0, "f64": 1, "f32": 2}
    segs = list(segments)
    if len(segs) > 8:
        raise ValueError("at most 8 assembler segments per launch")
    pad = lambda xs, v=0: list(xs) + [v] * (8 - len(xs))  # noqa: E731
    buf = struct.pack("i", len(segs)) + struct.pack("8i", *pad([kinds[s[0]] for s in segs]))
    buf += b"\0" * 4  # align pointer array to 8
    buf += struct.pack("8Q", *pad([s[1].data_ptr() for s in segs]))
    buf += struct.pack("8i", *pad([s[2] for s in segs])) + struct.pack("8i", *pad([s[3] for s in segs]))
    buf += struct.pack("8i", *pad([s[4] for s in segs]))
    size = _native.hip_lib().ptg_asm_desc_size()
    buf += b"\0" * (size - len(buf))
    cbuf = ctypes.create_string_buffer(buf, len(buf))
    hip("ptg_assemble_features", ctypes.addressof(cbuf), n, D, ptr(out))
    return out


def center_norms(C: torch.Tensor) -> torch.Tensor:
    k, Dm = C.shape
    if not on_device(C):
        return (C.double() ** 2).sum(1).float()
    cn = torch.empty(k, dtype=torch.float32, device=C.device)
    hip("ptg_center_norms", ptr(C), k, Dm, ptr(cn))
    return cn


KMEANS_DMAX = 576  # KM_DMAX in ml.hip: above it the kernels tile the feature dimension through LDS


def kmeans_assign_accum(X, C, assign=None, sums=None, counts=None, cost=None, weights=None, mind=None, cn=None,
                        done=None):
    """Fused k-means assignment: argmin_c ||x - c||^2 per row (-> assign, mind) and per-cluster
    sums / counts / cost accumulation.  ``done``: device flag that makes the launch a no-op."""
    n, D = X.shape
    k = C.shape[0]
    if not on_device(X):
        if done is not None and int(done.reshape(-1)[0]):
            return
        Xd, Cd = X.double(), C.double()
        d = (Xd * Xd).sum(1)[:, None] - 2 * Xd @ Cd.t() + (Cd * Cd).sum(1)[None, :]
        d = d.clamp_min(0)
        best, arg = d.min(1)
        if assign is not None:
            assign.copy_(arg.to(assign.dtype))
        if mind is not None:
            mind.copy_(best.to(mind.dtype))
        w = torch.ones(n, dtype=torch.float64, device=X.device) if weights is None else weights.double()
        if sums is not None:
            sums.index_add_(0, arg, (X.double() * w[:, None]).to(sums.dtype))
            counts.index_add_(0, arg, w.to(counts.dtype))
        if cost is not None:
            cost += (best * w).sum().to(cost.dtype)
        return
    if cn is None:
        cn = center_norms(C)
    hip("ptg_kmeans_assign_accum", ptr(X), ptr(C), ptr(cn), n, D, k, ptr(assign), ptr(sums), ptr(counts), ptr(cost),
        ptr(weights), ptr(mind), ptr(done))


def kmeans_update(sums, counts, C, moved, cn=None, done=None):
    """C = sums / counts (empty clusters keep their center); moved = max squared shift; sums and
    counts are zeroed for the next iteration (device); cn = new squared center norms."""
    k, D = C.shape
    if not on_device(C):
        newc = torch.where(counts[:, None] > 0, sums / counts.clamp_min(1e-30)[:, None], C)
        moved.fill_(float(((newc - C) ** 2).sum(1).max()))
        C.copy_(newc)
        if cn is not None:
            cn.copy_(center_norms(C))
        sums.zero_()
        counts.zero_()
        return
    hip("ptg_kmeans_update", ptr(sums), ptr(counts), ptr(C), ptr(cn), k, D, ptr(moved), ptr(done))


def kmeans_check(moved, tol2: float, state):
    """state[0] = done (moved <= tol2), state[1] += 1; moved reset — on the device, no readback."""
    if not on_device(moved):
        if not int(state[0]):
            state[1] += 1
            if float(moved[0]) <= tol2:
                state[0] = 1
        moved.zero_()
        return
    hip("ptg_kmeans_check", ptr(moved), float(tol2), ptr(state))


def silhouette_sum(X, assign, k: int):
    """Sum over points of Spark's squared-Euclidean silhouette coefficient (+ per-cluster stats)."""
    n, D = X.shape
    dev = X.device
    S = torch.zeros((k, D), dtype=torch.float32, device=dev)
    Q = torch.zeros(k, dtype=torch.float32, device=dev)
    cnt = torch.zeros(k, dtype=torch.float32, device=dev)
    if not on_device(X):
        a = assign.long()
        S.index_add_(0, a, X.float())
        Q.index_add_(0, a, (X.float() ** 2).sum(1))
        cnt.index_add_(0, a, torch.ones(n))
        return S, Q, cnt
    hip("ptg_cluster_stats", ptr(X), ptr(assign), n, D, ptr(S), ptr(Q), ptr(cnt))
    return S, Q, cnt


def silhouette_points(X, assign, S, Q, cnt) -> float:
    n, D = X.shape
    k = S.shape[0]
    if not on_device(X):
        Xd = X.double()
        xn = (Xd ** 2).sum(1)
        tot = cnt.double()[None, :] * xn[:, None] - 2 * Xd @ S.double().t() + Q.double()[None, :]
        a_idx = assign.long()
        own_n = cnt.double()[a_idx]
        a = torch.where(own_n > 1, tot.gather(1, a_idx[:, None]).squeeze(1) / (own_n - 1).clamp_min(1), torch.zeros(n, dtype=torch.float64))
        other = tot / cnt.double().clamp_min(1)[None, :]
        other[torch.arange(n), a_idx] = math.inf
        other[:, cnt <= 0] = math.inf
        b = other.min(1).values
        m = torch.maximum(a, b)
        s = torch.where((own_n > 1) & torch.isfinite(b) & (m > 0), (b - a) / m, torch.zeros_like(a))
        return float(s.sum())
    out = torch.zeros(1, dtype=torch.float64, device=X.device)
    hip("ptg_silhouette", ptr(X), ptr(assign), ptr(S), ptr(Q), ptr(cnt), n, D, k, ptr(out))
    return float(out.item())


# ------------------------------------------------------------------------------------------------
# group keys of any column types (csrc/kernels/dfkey.hip): exact multi-column / nullable keys
# ------------------------------------------------------------------------------------------------
KT_CODE = 5  # dictionary codes (int32, < 0 = null)
KMAX = 8


class _PackDesc(ctypes.Structure):
    _fields_ = [("ncols", ctypes.c_int), ("u", ctypes.c_void_p * KMAX), ("ok", ctypes.c_void_p * KMAX),
                ("lut", ctypes.c_void_p * KMAX), ("nlut", ctypes.c_long * KMAX), ("lo", ctypes.c_uint64 * KMAX),
                ("nullcode", ctypes.c_uint64 * KMAX), ("shift", ctypes.c_int * KMAX), ("bits", ctypes.c_int * KMAX),
                ("type", ctypes.c_int * KMAX)]


class _UnpackOut(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p * KMAX), ("valid", ctypes.c_void_p * KMAX)]


AMAX = 16


class _FinDesc(ctypes.Structure):
    _fields_ = [("nout", ctypes.c_int), ("fn", ctypes.c_int * AMAX), ("type", ctypes.c_int * AMAX),
                ("s", ctypes.c_void_p * AMAX), ("c", ctypes.c_void_p * AMAX), ("mn", ctypes.c_void_p * AMAX),
                ("mx", ctypes.c_void_p * AMAX), ("out", ctypes.c_void_p * AMAX), ("valid", ctypes.c_void_p * AMAX)]


def _check_struct_sizes() -> None:
    lib = _native.hip_lib()
    for name, st in (("ptg_key_desc_size", _PackDesc), ("ptg_unpack_out_size", _UnpackOut),
                     ("ptg_fin_desc_size", _FinDesc)):
        if getattr(lib, name)() != ctypes.sizeof(st):
            raise RuntimeError(f"{name}: host struct layout {ctypes.sizeof(st)} != device {getattr(lib, name)()}")


_STRUCTS_OK = [False]


KEY_ORDERABLE, KEY_RAW, KEY_RAW_TO_ORDERABLE = 0, 1, 2


def key_prep(data: torch.Tensor, kt: int, valid: torch.Tensor | None, need_ok: bool, stats: torch.Tensor,
             mode: int = KEY_ORDERABLE):
    """One column -> (orderable u64 keys in an int64 tensor, per-row valid flags u8 or None); its
    (min, max, null count) go into ``stats`` (3 int64 on the device, u64 bit patterns).
    ``mode`` KEY_RAW: raw canonical keys instead (what hash aggregation takes: never the tables'
    INT64_MIN empty marker except for that int64 value itself); KEY_RAW_TO_ORDERABLE: ``data`` holds
    raw canonical int64 keys of type ``kt``, converted to the orderable form."""
    if not _STRUCTS_OK[0]:
        _check_struct_sizes()
        _STRUCTS_OK[0] = True
    n = data.numel()
    d = data.view(torch.uint8) if data.dtype == torch.bool else data.contiguous()
    v = None if valid is None else (valid.view(torch.uint8) if valid.dtype == torch.bool else valid.contiguous())
    u = torch.empty(n, dtype=torch.int64, device=data.device)
    ok = torch.empty(n, dtype=torch.uint8, device=data.device) if need_ok else None
    hip("ptg_key_prep", ptr(d), kt, int(mode), ptr(v), n, ptr(u), ptr(ok), ptr(stats))
    return u, ok


def key_pack(cols, n: int, device) -> torch.Tensor:
    """``cols``: dicts with u, ok, lut (sorted distinct u or None), lo, nullcode, shift, bits, type."""
    D_ = _PackDesc()
    D_.ncols = len(cols)
    for j, c in enumerate(cols):
        D_.u[j] = c["u"].data_ptr()
        D_.ok[j] = c["ok"].data_ptr() if c["ok"] is not None else None
        D_.lut[j] = c["lut"].data_ptr() if c["lut"] is not None else None
        D_.nlut[j] = c["lut"].numel() if c["lut"] is not None else 0
        D_.lo[j], D_.nullcode[j] = c["lo"], c["nullcode"]
        D_.shift[j], D_.bits[j], D_.type[j] = c["shift"], c["bits"], c["type"]
    out = torch.empty(n, dtype=torch.int64, device=device)
    hip("ptg_key_pack", ctypes.addressof(D_), n, ptr(out))
    return out, D_


def key_unpack(keys: torch.Tensor, desc, outs: list) -> None:
    """``outs``: per column (data tensor of the column's type, valid u8 tensor or None)."""
    O = _UnpackOut()
    for j, (d, v) in enumerate(outs):
        O.data[j] = d.data_ptr()
        O.valid[j] = v.data_ptr() if v is not None else None
    hip("ptg_key_unpack", ptr(keys), keys.numel(), ctypes.addressof(desc), ctypes.addressof(O))


AF = {"rows": 0, "count": 1, "sum_int": 2, "sum": 3, "avg": 4, "min": 5, "max": 6}


def agg_finalize(rows: torch.Tensor, specs: list) -> None:
    """``specs``: (fn name, output KT type, s, c, mn, mx, out tensor, valid u8 tensor or None)."""
    for i in range(0, len(specs), AMAX):
        F = _FinDesc()
        part = specs[i:i + AMAX]
        F.nout = len(part)
        for j, (fn, kt, s, c, mn, mx, out, valid) in enumerate(part):
            F.fn[j], F.type[j] = AF[fn], kt
            F.s[j], F.c[j], F.mn[j], F.mx[j] = ptr(s), ptr(c), ptr(mn), ptr(mx)
            F.out[j], F.valid[j] = out.data_ptr(), ptr(valid)
        hip("ptg_agg_finalize", ptr(rows), rows.numel(), ctypes.addressof(F))


def iota_f64(n: int, device) -> torch.Tensor:
    out = torch.empty(n, dtype=torch.float64, device=device)
    hip("ptg_iota_f64", ptr(out), n)
    return out


def f64_to_i64(x: torch.Tensor) -> torch.Tensor:
    out = torch.empty(x.numel(), dtype=torch.int64, device=x.device)
    hip("ptg_f64_to_i64", ptr(x.contiguous()), ptr(out), x.numel())
    return out


def distinct_raw(raw: torch.Tensor) -> torch.Tensor:
    """Distinct raw canonical keys (unordered): hash aggregation without value columns."""
    if raw.numel() == 0:
        return raw
    return hash_agg(raw, [], [], est_keys=estimate_distinct(raw) if raw.numel() >= 65536 else None)[0]


def sorted_orderable(raw: torch.Tensor, kt: int) -> torch.Tensor:
    """Raw canonical keys of type ``kt`` -> their orderable forms, radix-sorted."""
    if raw.numel() == 0:
        return raw
    st = torch.empty(3, dtype=torch.int64, device=raw.device)
    u, _ = key_prep(raw, kt, None, False, st, mode=KEY_RAW_TO_ORDERABLE)
    sk, _ = radix_sort_u64(u, None, 0, _U64)
    return sk


def rr_part(n: int, rank: int, world: int, device) -> torch.Tensor:
    part = torch.empty(n, dtype=torch.int32, device=device)
    hip("ptg_rr_part", n, rank, world, ptr(part))
    return part


def part_override(part: torch.Tensor, flag: torch.Tensor, value: int) -> None:
    f = flag.view(torch.uint8) if flag.dtype == torch.bool else flag.contiguous()
    hip("ptg_part_override", ptr(part), ptr(f), part.numel(), int(value))
