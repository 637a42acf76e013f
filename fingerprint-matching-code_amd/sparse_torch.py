"""Batched CSR / CSC containers with the reference's interface (src/sparse_torch/csx_matrix.py).

``CSRMatrix3d`` / ``CSCMatrix3d`` hold one (indices, indptr, data) triple for a (b, h, w) batch:
int64 indices, an int64 indptr of length b*h+1 (CSR) or b*w+1 (CSC) with GLOBAL offsets into
indices/data (csx_matrix.py:20-93).  Constructors accept a list of scipy sparse matrices or an
[indices, indptr, data] list, as in the reference.

The products run through ``libfpm_hip.so``: device tensors use the HIP kernels
(``fpm_csr_dot_csc_to_dense``, ``fpm_dense_dot_csc_to_dense``, ``fpm_csr_dot_diag_to_csr``), CPU
tensors the library's host twins -- the same split as the reference's extension, which runs
csr x csc -> csr and the diagonal product on the CPU (sparse_dot.cpp:50-140, 228-255) and the
dense-output products on the GPU only (csx_matrix.py:484-500).
"""
import ctypes

import numpy as np
import scipy.sparse as ssp
import torch

from . import _lib

_DT = {torch.float32: 0, torch.float64: 2, torch.float16: 3}


def _code(t, host=False):
    if t.dtype not in _DT or (host and t.dtype == torch.float16):
        raise _lib.FpmError("sparse op: unsupported data dtype %s" % t.dtype)
    return _DT[t.dtype]


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _same_device(dev, *ts):
    """Every operand of one launch on ``dev`` (a host pointer handed to a kernel would fault)."""
    for t in ts:
        if t.device != dev:
            raise _lib.FpmError("sparse op: operand on %s, expected %s" % (t.device, dev))


def _max(inp):
    if isinstance(inp, np.ndarray):
        return np.max(inp)
    if isinstance(inp, torch.Tensor):
        return torch.max(inp)
    raise ValueError('Data type {} not understood.'.format(type(inp)))


class CSXMatrix3d:
    """Common part of the CSR/CSC batch containers (csx_matrix.py:20-331)."""

    def __init__(self, inp, shape, device=None):
        if type(inp) == list and len(inp) > 0 and isinstance(inp[0], ssp.spmatrix):
            self.indices, self.indptr, self.data, self.shape = self._from_ssp(inp, shape, device)
        elif type(inp) == list:
            self.indices, self.indptr, self.data, self.shape = self._from_tensors(*inp, shape=shape, device=device)
        else:
            raise ValueError('Data type {} not understood.'.format(type(inp)))

    # -- construction ----------------------------------------------------------------------
    def _from_ssp(self, mats, shape, device):
        assert len(shape) == 3, 'Only 3-dimensional tensor (bxhxw) is supported'
        ind, ptr, dat = [], [], []
        off = 0
        for b in range(shape[0]):
            m = mats[b]
            m.eliminate_zeros()
            sp = (m.tocsc() if self.sptype == 'csc' else m.tocsr()).astype(m.dtype)
            ind.append(sp.indices)
            ptr.append(sp.indptr[:-1] + off)
            dat.append(sp.data)
            off += sp.indptr[-1]
        ptr.append(np.array([off]))
        return self._from_tensors(np.concatenate(ind), np.concatenate(ptr), np.concatenate(dat), shape=shape,
                                  device=device)

    @staticmethod
    def _from_tensors(ind, indp, data, shape, device=None):
        if isinstance(ind, torch.Tensor) and device is None:
            device = ind.device
        cvt = lambda a: (a.to(torch.int64).to(device) if isinstance(a, torch.Tensor)
                         else torch.tensor(a, dtype=torch.int64, device=device))
        d = data.to(device) if isinstance(data, torch.Tensor) else torch.tensor(data, device=device)
        return cvt(ind), cvt(indp), d, tuple(shape)

    # -- batch access ----------------------------------------------------------------------
    def _clen(self):
        return self.shape[1] if self.sptype == 'csr' else self.shape[2]

    def get_batch(self, item):
        if type(item) != int:
            raise IndexError('Only int indices is currently supported.')
        n = self._clen()
        ptr = self.indptr[item * n:(item + 1) * n + 1].clone()
        lo, hi = int(ptr[0]), int(ptr[-1])
        return self.indices[lo:hi].clone(), ptr - ptr[0], self.data[lo:hi].clone()

    def __getitem__(self, item):
        if isinstance(item, int):
            i, p, d = self.get_batch(item)
            return self.__class__([i, p, d], shape=[1] + list(self.shape[1:3]))
        if isinstance(item, slice):
            rng = range(*item.indices(self.shape[0]))
            parts = [self.get_batch(b) for b in rng]
            return _stack(self.__class__, parts, (len(rng),) + tuple(self.shape[1:3]), self.device)
        raise ValueError('Index type {} not supported.'.format(type(item)))

    def __len__(self):
        return self.shape[0]

    @property
    def device(self):
        return self.indices.device

    @property
    def sptype(self):
        raise NotImplementedError

    def transpose(self, keep_type=False):
        raise NotImplementedError

    # -- conversions -----------------------------------------------------------------------
    def to(self, tgt):
        if isinstance(tgt, torch.device):
            return self.__class__([x.to(tgt) for x in self.as_list()], self.shape)
        if isinstance(tgt, torch.dtype):
            return self.__class__([self.indices, self.indptr, self.data.to(tgt)], self.shape)
        raise ValueError('Data type not understood.')

    def cuda(self):
        return self.__class__([x.cuda() for x in self.as_list()], self.shape)

    def cpu(self):
        return self.__class__([x.cpu() for x in self.as_list()], self.shape)

    def numpy(self):
        return np.stack([m.toarray() for m in self.as_ssp()], axis=0)

    def as_list(self, mask=None):
        attrs = [self.indices, self.indptr, self.data]
        return attrs if mask is None else [a for m, a in zip(mask, attrs) if m]

    def as_ssp(self):
        ctor = ssp.csr_matrix if self.sptype == 'csr' else ssp.csc_matrix
        out = []
        for b in range(self.shape[0]):
            i, p, d = self.get_batch(b)
            out.append(ctor((d.cpu().numpy(), i.cpu().numpy(), p.cpu().numpy()), shape=self.shape[1:3]))
        return out

    def _coo(self):
        """(batch, row, col) of every stored entry, in storage order."""
        n = self._clen()
        counts = (self.indptr[1:] - self.indptr[:-1]).to(torch.long)
        slot = torch.repeat_interleave(torch.arange(self.shape[0] * n, device=self.device), counts)
        bidx, comp = slot // n, slot % n
        if self.sptype == 'csr':
            return bidx, comp, self.indices
        return bidx, self.indices, comp

    def as_sparse_torch(self):
        b, r, c = self._coo()
        return torch.sparse_coo_tensor(torch.stack([b, r, c]), self.data, self.shape)

    def shape_eq(self, other):
        return all(s == o for s, o in zip(self.shape, other.shape))

    def diagonal(self):
        assert self.shape[1] == self.shape[2], 'Only square matrix has diagonals'
        out = torch.zeros((self.shape[0], self.shape[1]), device=self.device)
        b, r, c = self._coo()
        on = r == c
        # first stored occurrence per (b, i) wins, as in the reference's nonzero()[0]
        key = b[on] * self.shape[1] + r[on]
        vals = self.data[on]
        pos = torch.arange(key.numel(), device=self.device)
        first = torch.full((self.shape[0] * self.shape[1],), key.numel(), dtype=torch.long, device=self.device)
        first.scatter_reduce_(0, key, pos, reduce='amin')
        hit = first < key.numel()
        out.view(-1)[hit] = vals[first[hit]].to(out.dtype)
        return out

    @classmethod
    def from_dense(cls, dense_tensor, device=None):
        assert len(dense_tensor.shape) == 3, 'input tensor must be 3-dimensional'
        if device is None:
            device = dense_tensor.device
        if cls.sptype.fget(None) == 'csr':
            src = dense_tensor
        else:
            src = dense_tensor.transpose(1, 2)
        nz = src.nonzero(as_tuple=False)            # row-major order of the compressed view
        B, n = src.shape[0], src.shape[1]
        counts = torch.bincount(nz[:, 0] * n + nz[:, 1], minlength=B * n)
        indp = torch.zeros(B * n + 1, dtype=torch.int64, device=device)
        indp[1:] = torch.cumsum(counts, 0).to(device)
        data = src[nz[:, 0], nz[:, 1], nz[:, 2]]
        return cls([nz[:, 2].to(device), indp, data.to(device)], tuple(dense_tensor.shape), device)


def _stack(cls, parts, shape, device):
    ind, ptr, dat = [], [], []
    off = torch.zeros((), dtype=torch.int64, device=device)
    for i, p, d in parts:
        ind.append(i)
        ptr.append(p[:-1] + off)
        dat.append(d)
        off = off + p[-1]
    ptr.append(off.view(1))
    return cls([torch.cat(ind), torch.cat(ptr), torch.cat(dat)], shape=shape)


class CSCMatrix3d(CSXMatrix3d):
    """csx_matrix.py:333-382."""

    def __init__(self, inp, shape=None, device=None):
        if type(inp) == list and len(inp) > 0 and isinstance(inp[0], ssp.spmatrix):
            mx = [max(s.shape[0] for s in inp), max(s.shape[1] for s in inp)]
            if shape is None:
                shape = tuple([len(inp)] + mx)
            else:
                assert shape[0] == len(inp)
                assert shape[1] <= mx[0]
                assert shape[2] <= mx[1]
        elif type(inp) == list:
            assert shape is not None
            col = (len(inp[1]) - 1) // shape[0]
            if len(inp[0]) > 0:
                assert shape[1] >= _max(inp[0])
            assert shape[2] == col
        super().__init__(inp, shape, device)

    @property
    def sptype(self):
        return 'csc'

    def transpose(self, keep_type=False):
        if not keep_type:
            s = list(self.shape)
            return CSRMatrix3d(self.as_list(), shape=[s[0], s[2], s[1]], device=self.device)
        return CSCMatrix3d([m.transpose().tocoo().astype(m.dtype) for m in self.as_ssp()], device=self.device)

    def Tdot(self, other, *args, **kwargs):
        return dot(self.transpose(), other, *args, **kwargs)


class CSRMatrix3d(CSXMatrix3d):
    """csx_matrix.py:385-465."""

    def __init__(self, inp, shape=None, device=None):
        if type(inp) == list and len(inp) > 0 and isinstance(inp[0], ssp.spmatrix):
            mx = [max(s.shape[0] for s in inp), max(s.shape[1] for s in inp)]
            if shape is None:
                shape = tuple([len(inp)] + mx)
            else:
                assert shape[0] == len(inp)
                assert shape[1] <= mx[0]
                assert shape[2] <= mx[1]
        elif type(inp) == list:
            assert shape is not None
            row = (len(inp[1]) - 1) // shape[0]
            assert shape[1] == row
            if len(inp[0]) > 0:
                assert shape[2] >= _max(inp[0])
        super().__init__(inp, shape, device)

    @property
    def sptype(self):
        return 'csr'

    def transpose(self, keep_type=False):
        if not keep_type:
            s = list(self.shape)
            return CSCMatrix3d(self.as_list(), shape=[s[0], s[2], s[1]], device=self.device)
        return CSRMatrix3d([m.transpose().tocoo().astype(m.dtype) for m in self.as_ssp()], device=self.device)

    def dot(self, other, *args, **kwargs):
        return dot(self, other, *args, **kwargs)

    def dotdiag(self, other):
        """CSR x diag(other[b]) (csx_matrix.py:434-441 -> sparse_dot.csr_dot_diag_to_csr)."""
        assert self.shape[0] == other.shape[0], 'Batch size mismatch'
        assert self.shape[2] == other.shape[1], 'Matrix shape mismatch'
        B, h, w = self.shape
        other = other.to(self.data.dtype).contiguous()
        _same_device(self.data.device, self.indices, self.indptr, other)
        out = torch.zeros_like(self.data)
        if self.data.is_cuda:
            _lib.call("fpm_csr_dot_diag_to_csr", _code(self.data), _p(self.indices), _p(self.indptr),
                      _p(self.data.contiguous()), _p(other), B, h, w, _p(out), _stream(self.device))
        else:
            _lib.call("fpm_csr_dot_diag_to_csr_host", _code(self.data, True), _p(self.indices), _p(self.indptr),
                      _p(self.data.contiguous()), _p(other), B, h, w, _p(out))
        return CSRMatrix3d([self.indices.clone(), self.indptr.clone(), out], shape=self.shape)


def _csr_dot_csc_host(t1, t2, B, out_h, out_w):
    _same_device(torch.device('cpu'), t1.indices, t1.indptr, t1.data, t2.indices, t2.indptr, t2.data)
    lib = _lib.load()
    code = _code(t1.data, True)
    a = [_p(x) for x in (t1.indices, t1.indptr, t1.data.contiguous(), t2.indices, t2.indptr,
                         t2.data.to(t1.data.dtype).contiguous())]
    ptr = torch.zeros(B * out_h + 1, dtype=torch.int64)
    nnz = lib.fpm_csr_dot_csc_to_csr_host(code, *a, B, out_h, out_w, _p(ptr), 0, None, None)
    if nnz < 0:
        raise _lib.FpmError(lib.fpm_last_error().decode())
    ind = torch.zeros(max(nnz, 1), dtype=torch.int64)
    dat = torch.zeros(max(nnz, 1), dtype=t1.data.dtype)
    lib.fpm_csr_dot_csc_to_csr_host(code, *a, B, out_h, out_w, _p(ptr), nnz, _p(ind), _p(dat))
    return ind[:nnz], ptr, dat[:nnz]


def dot(t1, t2, dense_output=False):
    """CSR/dense x CSC (csx_matrix.py:468-503)."""
    assert t1.shape[0] == t2.shape[0], 'Batch size mismatch'
    B = t1.shape[0]
    assert t1.shape[2] == t2.shape[1], 'Matrix size mismatch'
    out_h, out_w, t1_w = t1.shape[1], t2.shape[2], t1.shape[2]
    if type(t1) == CSRMatrix3d and type(t2) == CSCMatrix3d:
        if t1.indptr.device == torch.device('cpu'):
            ret = CSRMatrix3d(list(_csr_dot_csc_host(t1, t2, B, out_h, out_w)), shape=(B, out_h, out_w))
            return ret.numpy() if dense_output else ret
        if not dense_output:
            raise NotImplementedError('Sparse dot product result in CUDA is not implemented.')
        _same_device(t1.data.device, t1.indices, t1.indptr, t2.indices, t2.indptr, t2.data)
        out = torch.empty(B, out_h, out_w, dtype=t1.data.dtype, device=t1.device)
        _lib.call("fpm_csr_dot_csc_to_dense", _code(t1.data), _p(t1.indices), _p(t1.indptr),
                  _p(t1.data.contiguous()), _p(t2.indices), _p(t2.indptr), _p(t2.data.to(t1.data.dtype).contiguous()),
                  B, out_h, out_w, _p(out), _stream(t1.device))
        return out
    if type(t1) == torch.Tensor and type(t2) == CSCMatrix3d:
        if t1.device != torch.device('cpu') and dense_output:
            t1c = t1.contiguous()
            _same_device(t1.device, t2.indices, t2.indptr, t2.data)
            out = torch.empty(B, out_h, out_w, dtype=t1.dtype, device=t1.device)
            _lib.call("fpm_dense_dot_csc_to_dense", _code(t1c), _p(t1c), _p(t2.indices), _p(t2.indptr),
                      _p(t2.data.to(t1.dtype).contiguous()), B, out_h, out_w, t1_w, _p(out), _stream(t1.device))
            return out
        raise NotImplementedError('Not implemented: dense * sparse CSC -> dense.')
    raise ValueError(f'Types of t1, t2 are not supported. Got type(t1)={type(t1)}, type(t2)={type(t2)}')


def concatenate(*mats, device=None):
    """Concatenate along the batch dimension (csx_matrix.py:506-540)."""
    device = mats[0].device if device is None else device
    cls, h, w = type(mats[0]), mats[0].shape[1], mats[0].shape[2]
    for m in mats:
        assert type(m) == cls, 'Matrix type inconsistent'
        assert m.shape[1] == h, 'Matrix shape inconsistent in dimension 1'
        assert m.shape[2] == w, 'Matrix shape inconsistent in dimension 2'
    parts = [(m.indices.to(device), m.indptr.to(device), m.data.to(device)) for m in mats]
    return _stack(cls, parts, (sum(m.shape[0] for m in mats), h, w), device)
