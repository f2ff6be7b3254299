"""Transformer modules (reference ``minitorch/modules_transfomer.py``).

``MultiHeadAttention(use_flash_attention=True)`` is the north-star caller: its
``self_attention`` hands the permuted ``[B, H, N, d]`` projections straight to
``q.flash_attention[_causal](k, v)`` (reference :154-175). The plain branch is the
unfused ``softmax(QKᵀ/√d) V`` composition (reference :177-193) and the fused-softmax
branch uses the HIP attention softmax (with the causal mask applied inside the kernel).

Fixes vs the reference: the ``use_flash_attention`` / ``use_fused_kernel`` flags reach
MultiHeadAttention from TransformerLayer and DecoderLM by keyword (reference :309-311,
:409-420 pass them positionally into the wrong slots); position embeddings are sized by
``n_positions`` (reference :408 uses ``n_vocab``).
"""
from __future__ import annotations

import numpy as np

from .module import Module
from .modules_basic import Dropout, Embedding, FusedLayerNorm, LayerNorm1d, Linear
from .nn import GELU, softmax
from .tensor_functions import tensor, tensor_from_numpy

# Small host-built index tensors the model makes on every forward (the [B] key-padding lengths
# of the flash path, the [1, T] position ids): cached by value, so a training loop that feeds
# the same shapes does not copy host memory to the device in every layer (each synchronous
# host-to-device copy also waits for the work already queued on the stream)
_INDEX_CACHE: dict = {}


def _kv_tensor(kv_len, batch_size: int, backend):
    from .tensor import Tensor
    if isinstance(kv_len, Tensor):  # already a device tensor (e.g. a graph-captured step's fixed input)
        if kv_len.size != batch_size:
            raise ValueError(f"kv_len has {kv_len.size} entries for a batch of {batch_size}")
        return kv_len
    a = np.ascontiguousarray(np.asarray(kv_len, dtype=datatype).reshape(batch_size))
    key = ("kv", id(backend), a.tobytes())
    t = _INDEX_CACHE.get(key)
    if t is None:
        if len(_INDEX_CACHE) > 64:
            _INDEX_CACHE.clear()
        t = _INDEX_CACHE[key] = tensor_from_numpy(a, backend=backend)
    return t


def _positions(seq_len: int, backend):
    key = ("pos", id(backend), seq_len)
    t = _INDEX_CACHE.get(key)
    if t is None:
        if len(_INDEX_CACHE) > 64:
            _INDEX_CACHE.clear()
        t = _INDEX_CACHE[key] = tensor([[float(i) for i in range(seq_len)]], backend=backend)
    return t

datatype = np.float32


class MultiHeadAttention(Module):
    def __init__(self, n_embd: int, n_head: int, causal: bool = False, p_dropout: float = 0.1,
                 bias: bool = True, backend=None, use_fused_kernel: bool = False,
                 use_flash_attention: bool = False):
        super().__init__()
        self.backend = backend
        self.n_embd = n_embd
        self.n_head = n_head
        self.causal = causal
        self.attn_hidden_dim = n_embd // n_head
        self.q_projection = Linear(n_embd, n_embd, bias, backend)
        self.k_projection = Linear(n_embd, n_embd, bias, backend)
        self.v_projection = Linear(n_embd, n_embd, bias, backend)
        self.out_projection = Linear(n_embd, n_embd, bias, backend)
        self.dropout = Dropout(p_dropout)
        self.use_fused_kernel = use_fused_kernel
        self.use_flash_attention = use_flash_attention

    def create_causal_mask(self, bs, nh, seq_len):
        """Additive -FLT_MAX·triu(1) mask (reference :63-71), [1, 1, T, T] broadcast."""
        mask = -np.finfo(datatype).max * np.triu(np.ones((1, 1, seq_len, seq_len), dtype=datatype), 1)
        return tensor_from_numpy(mask, backend=self.backend)

    def project_to_query_key_value(self, x):
        batch_size, seq_len, n_embd = x.shape
        flat = x.view(batch_size * seq_len, n_embd)
        shp = (batch_size, seq_len, self.n_head, self.attn_hidden_dim)
        q = self.q_projection(flat).view(*shp).permute(0, 2, 1, 3)
        k4 = self.k_projection(flat).view(*shp)
        kT = k4.permute(0, 2, 3, 1)
        k = k4.permute(0, 2, 1, 3)
        v = self.v_projection(flat).view(*shp).permute(0, 2, 1, 3)
        return q, k, kT, v

    def create_padding_mask(self, kv_len, seq_len):
        """The reference's key-padding contract (src/softmax_kernel.cu:26-33: attn_mask
        [B, to_len], 0 for tokens, -inf for padding) as an additive [B, 1, 1, T] mask."""
        kv = np.asarray(kv_len).reshape(-1, 1, 1, 1)
        mask = np.where(np.arange(seq_len)[None, None, None, :] < kv, 0.0, -np.inf).astype(datatype)
        return tensor_from_numpy(mask, backend=self.backend)

    def self_attention(self, q, kT, v, kv_len=None):
        """``kT`` is the [B,H,d,N] transpose, or the [B,H,N,d] keys on the flash path.
        ``kv_len``: optional per-batch-row count of valid (non-padding) keys: the flash path
        masks keys >= kv_len[b] in the kernel (mt_flash_attn_*_varlen); the other branches add
        the equivalent [B, to_len] padding mask."""
        batch_size, num_head, queries_len, q_dim = q.shape
        scale = self.attn_hidden_dim ** 0.5
        if self.use_flash_attention:
            kv = None if kv_len is None else _kv_tensor(kv_len, batch_size, self.backend)
            result = (q.flash_attention_causal(kT, v, kv_len=kv) if self.causal
                      else q.flash_attention(kT, v, kv_len=kv))
        elif self.use_fused_kernel:
            scores = (q @ kT) / scale
            if kv_len is None:
                result = (scores.attn_softmax(None, mask_future=True) if self.causal
                          else scores.attn_softmax(None)) @ v
            else:
                mask = self.create_padding_mask(kv_len, queries_len)
                if self.causal:
                    mask = mask + self.create_causal_mask(batch_size, num_head, queries_len)
                result = scores.attn_softmax(mask) @ v
        else:
            scores = (q @ kT) / scale
            if self.causal:
                scores = scores + self.create_causal_mask(batch_size, num_head, queries_len)
            if kv_len is not None:
                scores = scores + self.create_padding_mask(kv_len, queries_len)
            result = softmax(scores, dim=3) @ v
        result = result.permute(0, 2, 1, 3).contiguous()
        return result.view(batch_size, queries_len, self.n_embd)

    def forward(self, x, kv_len=None):
        batch_size, seq_len, n_embd = x.shape
        q, k, kT, v = self.project_to_query_key_value(x)
        attn = self.self_attention(q, k if self.use_flash_attention else kT, v, kv_len)
        return self.out_projection(attn.view(batch_size * seq_len, n_embd)).view(batch_size, seq_len, n_embd)


class FeedForward(Module):
    def __init__(self, n_embd: int, middle_dim: int = 256, p_dropout: float = 0.1, bias: bool = True,
                 backend=None):
        super().__init__()
        self.linear_in = Linear(n_embd, middle_dim, bias=bias, backend=backend)
        self.linear_out = Linear(middle_dim, n_embd, bias=bias, backend=backend)
        self.dropout = Dropout(p_dropout)

    def forward(self, x):
        batch_size, seq_len, n_embd = x.shape
        flat = x.view(batch_size * seq_len, n_embd)
        be = x.backend
        if (getattr(be, "bias_gelu_fw", None) is not None and self.linear_in.bias is not None
                and x._tensor.on_device):
            # linear_in's bias add and the GELU as one kernel each way (BiasGelu)
            from .tensor_functions import BiasGelu
            h = BiasGelu.apply(flat @ self.linear_in.weights.value, self.linear_in.bias.value)
        else:
            h = GELU(self.linear_in(flat))
        return self.dropout(self.linear_out(h)).view(batch_size, seq_len, n_embd)


class TransformerLayer(Module):
    """Pre-LN transformer block (reference :279-362)."""

    def __init__(self, n_embd: int, n_head: int, p_dropout: float = 0.1, ln_eps: float = 1e-8,
                 bias: bool = True, backend=None, use_fused_kernel: bool = False,
                 use_flash_attention: bool = False, causal: bool = True):
        super().__init__()
        self.attention = MultiHeadAttention(n_embd, n_head, causal=causal, p_dropout=p_dropout,
                                            bias=bias, backend=backend,
                                            use_fused_kernel=use_fused_kernel,
                                            use_flash_attention=use_flash_attention)
        self.ff = FeedForward(n_embd, 256, p_dropout, bias, backend)
        self.use_fused_kernel = use_fused_kernel
        if use_fused_kernel:
            self.ln_1 = FusedLayerNorm(n_embd, backend)
            self.ln_2 = FusedLayerNorm(n_embd, backend)
        else:
            self.ln_1 = LayerNorm1d(n_embd, ln_eps, backend)
            self.ln_2 = LayerNorm1d(n_embd, ln_eps, backend)

    def forward(self, x, kv_len=None):
        batch_size, seq_len, x_dim = x.shape
        a = self.ln_1(x.view(batch_size * seq_len, x_dim)).view(batch_size, seq_len, x_dim)
        a = self.attention(a, kv_len) + x
        h = self.ln_2(a.view(batch_size * seq_len, x_dim)).view(batch_size, seq_len, x_dim)
        return self.ff(h) + a


class DecoderLM(Module):
    """Decoder-only pre-LN LM with 4 TransformerLayers (reference :365-470)."""

    def __init__(self, n_vocab: int, n_embd: int, n_head: int, n_positions: int,
                 p_dropout: float = 0.1, ln_eps: float = 1e-5, bias: bool = True, backend=None,
                 use_fused_kernel: bool = False, use_flash_attention: bool = False, n_layer: int = 4):
        super().__init__()
        self.backend = backend
        self.n_embd = n_embd
        self.n_vocab = n_vocab
        self.n_layer = n_layer
        self.token_embeddings = Embedding(n_vocab, n_embd, backend)
        self.position_embeddings = Embedding(n_positions, n_embd, backend)
        for i in range(n_layer):
            setattr(self, f"t_layer_{i + 1}", TransformerLayer(
                n_embd, n_head, p_dropout, ln_eps, bias, backend,
                use_fused_kernel=use_fused_kernel, use_flash_attention=use_flash_attention))
        self.dropout = Dropout(p_dropout)
        self.lm_head = Linear(n_embd, n_vocab, bias, backend)
        self.use_fused_kernel = use_fused_kernel
        self.ln = FusedLayerNorm(n_embd, backend) if use_fused_kernel else LayerNorm1d(n_embd, ln_eps, backend)

    def forward(self, idx, kv_len=None):
        """kv_len: optional valid-token count per batch row of a right-padded batch (keys past
        it are masked in every layer's self-attention; with the causal mask and right padding
        this changes only the outputs at padding positions)."""
        batch_size, seq_len = idx.shape
        pos = _positions(seq_len, self.backend)
        h = self.token_embeddings(idx) + self.position_embeddings(pos).view(1, seq_len, self.n_embd)
        h = self.dropout(h)
        for i in range(self.n_layer):
            h = getattr(self, f"t_layer_{i + 1}")(h, kv_len)
        h = self.ln(h.view(batch_size * seq_len, self.n_embd))
        return self.lm_head(h).view(batch_size, seq_len, self.n_vocab)
