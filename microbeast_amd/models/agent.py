"""IMPALA-CNN agent with a flat per-cell masked multi-discrete head.

Same architecture, parameter names and initialisation as the reference
``Agent`` (reference model.py:112-220), so reference state_dicts load 1:1:

* ``network.{0,1,2}``: ConvSequence(conv3x3 -> maxpool(3,2,1) -> 2 residual
  blocks), channels 16/32/32 (model.py:77-107, 56-73);
* ``network.5``: Linear(32*ceil(h/8)*ceil(w/8), 256) after Flatten+ReLU,
  followed by ReLU (model.py:125-133);
* ``actor``: Linear(256, 78*h*w), orthogonal gain 0 (uniform initial policy);
  ``critic``: Linear(256, 1), orthogonal gain 1 (model.py:136-137).

Differences that fix reference defects: the encoder runs once per
call and feeds both heads (D7); device handling is real (D6); learning scores
actions against the observation they were sampled at (the caller aligns, D3).

Observations may be the compact uint32 bit planes (GPU engine / native env)
or the reference dense float (N, h, w, 27) layout.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import cell_head
from ..ops.encoder import HipEncoder, encode, encoder_params
from ..ops.head import SparseHead, sparse_sample, sparse_score
from ..ops.linear import linear, nhwc_weight
from ..ops.obs import bits_to_planes, dense_to_bits
from ..ops.pixconv import map_gather
from ..ops.tail import TailMaps, impala_tail

HIP_CHANNELS = (16, 32)  # conv widths the HIP trunk kernels are instantiated for




def layer_init(layer: nn.Module, std: float = math.sqrt(2), bias_const: float = 0.0) -> nn.Module:
    """reference model.py:24-27"""
    nn.init.orthogonal_(layer.weight, std)
    nn.init.constant_(layer.bias, bias_const)
    return layer


class ResidualBlock(nn.Module):
    """x + conv1(relu(conv0(relu(x)))) — reference model.py:56-73."""

    def __init__(self, channels: int):
        super().__init__()
        self.conv0 = nn.Conv2d(channels, channels, 3, padding=1)
        self.conv1 = nn.Conv2d(channels, channels, 3, padding=1)

    def forward(self, x):
        y = self.conv0(F.relu(x))
        y = self.conv1(F.relu(y))
        return x + y


class ConvSequence(nn.Module):
    """conv -> maxpool(3, 2, 1) -> res -> res — reference model.py:77-107."""

    def __init__(self, input_shape, out_channels: int):
        super().__init__()
        self._input_shape = tuple(input_shape)
        self._out_channels = out_channels
        self.conv = nn.Conv2d(input_shape[0], out_channels, 3, padding=1)
        self.res_block0 = ResidualBlock(out_channels)
        self.res_block1 = ResidualBlock(out_channels)

    def forward(self, x):
        x = self.conv(x)
        x = F.max_pool2d(x, kernel_size=3, stride=2, padding=1)
        x = self.res_block0(x)
        return self.res_block1(x)

    def get_output_shape(self):
        _c, h, w = self._input_shape
        return (self._out_channels, (h + 1) // 2, (w + 1) // 2)


class Agent(nn.Module):
    """Reference-compatible constructor: ``Agent(obs_space_shape, nvec, mapsize, device)``.

    ``obs_space_shape`` = (h, w, planes); ``nvec`` = the MultiDiscrete nvec list
    ([6,4,4,4,4,7,49] * h*w) or None to derive it from the map size.
    """

    accepts_abits = True  # evaluate(..., abits=): the acting step's active-cell bitmap

    def __init__(self, obs_space_shape=(16, 16, 27), nvec=None, mapsize=None, device="cpu",
                 channels=(16, 32, 32), hidden=256, compute_dtype=torch.bfloat16,
                 hip_kernels: bool = True):
        super().__init__()
        self.channels = tuple(channels)
        self.hip_kernels = hip_kernels
        self._hip_enc = None
        self._hip_head = None
        self.fp8_inference = False  # acting trunk on the fp8 MFMA convs (see HipEncoder)
        self._prepacked = False     # inference copy: derived weight buffers are current
        self._fc_cache = None
        h, w, c = obs_space_shape
        self.h, self.w, self.planes = h, w, c
        self.mapsize = mapsize if mapsize is not None else h * w
        self.nvec = list(nvec) if nvec is not None else list(cell_head.NVEC) * (h * w)
        assert sum(self.nvec) == cell_head.CELL * h * w, "flat head expects 78 logits per cell"
        shape = (c, h, w)
        seqs = []
        for oc in channels:
            cs = ConvSequence(shape, oc)
            shape = cs.get_output_shape()
            seqs.append(cs)
        self.network = nn.Sequential(
            *seqs, nn.Flatten(), nn.ReLU(),
            nn.Linear(shape[0] * shape[1] * shape[2], hidden), nn.ReLU())
        self.actor = layer_init(nn.Linear(hidden, sum(self.nvec)), std=0.0)
        self.critic = layer_init(nn.Linear(hidden, 1), std=1)
        self.compute_dtype = compute_dtype
        self._tail_maps = None
        for p in self.parameters():  # the HIP learner path writes grads into flat slots
            p._mbk_direct_grad = True
        self.to(device)

    # ------------------------------------------------------------ encoder
    def _planes(self, obs: torch.Tensor) -> torch.Tensor:
        if obs.dtype in (torch.int32, torch.uint32):
            return bits_to_planes(obs.reshape(-1, self.h * self.w), self.h, self.w, torch.float32,
                                  self.planes)
        return obs.reshape(-1, self.h, self.w, self.planes).permute(0, 3, 1, 2).float()

    def _autocast(self, t: torch.Tensor):
        enabled = t.is_cuda and self.compute_dtype in (torch.bfloat16, torch.float16)
        # no weight-cast cache: each weight is used once per forward, and cached
        # casts must not leak across hipGraph capture boundaries
        return torch.autocast("cuda", dtype=self.compute_dtype, enabled=enabled,
                              cache_enabled=False)

    def direct_grad_ok(self, device) -> bool:
        """the learner's backward writes every gradient into its flat slot (ops/tail.py,
        ops/encoder.py) -- the HIP path on a GPU"""
        return (self.hip_kernels and torch.device(device).type == "cuda"
                and all(c in HIP_CHANNELS for c in self.channels))

    def _use_hip(self, obs: torch.Tensor) -> bool:
        if not (self.hip_kernels and obs.is_cuda and obs.dtype == torch.int32):
            return False
        if not all(c in HIP_CHANNELS for c in self.channels):
            # no silent vendor-library fallback on the GPU: say what to do instead
            raise RuntimeError(
                f"HIP conv kernels exist for channel widths {HIP_CHANNELS}, this Agent has "
                f"{self.channels}; construct it with hip_kernels=False to run the PyTorch "
                f"(MIOpen) path instead")
        return True

    def _compact_obs(self, obs: torch.Tensor) -> torch.Tensor:
        """Reference-layout float one-hot obs (N, h, w, planes) on the GPU -> the uint32
        bit-plane form the HIP kernels read, so the reference API runs on the same kernels
        as the engine (not on MIOpen / hipBLASLt). Other inputs pass through unchanged."""
        if (self.hip_kernels and obs.is_cuda and obs.is_floating_point()
                and obs.shape[-1] == self.planes and self.planes <= 32):
            return dense_to_bits(obs.reshape(-1, self.h, self.w, self.planes))
        return obs

    def _rng(self, device) -> torch.Tensor:
        """Philox (seed, step) state for the reference API's on-device sampling."""
        r = getattr(self, "_api_rng", None)
        if r is None or r.device != device:
            seed = int(torch.randint(0, 2**31 - 1, (1,)).item())
            r = self._api_rng = torch.tensor([seed, 0], dtype=torch.int64, device=device)
        return r

    def _act_features(self, obs: torch.Tensor, value_out: torch.Tensor | None = None):
        """Acting forward with prepacked weights: conv trunk, then ONE fused launch for
        relu -> network.5 -> relu -> critic (fc.hip). Returns (f bf16 [N,256], value fp32);
        value_out: fp32 [N] the fused kernel writes the value into (no copy launch)."""
        from .. import _native as N
        n = obs.shape[0] if obs.dim() == 2 else obs.numel() // (self.h * self.w)
        fc = self.network[len(self.channels) + 2]
        # (network.5 + critic inside the trunk launch, mbk_trunk_tail_fc, measured 0.208 vs
        # 0.200 ms per 8192-env step and no gain under the learner: the separate launch)
        y = encode(obs.reshape(n, self.h * self.w), self._hip_enc,
                   encoder_params(self.network, len(self.channels)), False, prepacked=True,
                   value_out=value_out)
        if isinstance(y, tuple):
            return y
        I = y[0].numel()
        if fc.out_features not in (128, 256, 512):  # no fused kernel instance: cached GEMMs
            c = self._fc_cache
            f = F.relu(linear(F.relu(y.reshape(n, -1)), fc, cached=(c["w5"], c["b5"])))
            return f, linear(f, self.critic, cached=(c["wc"], c["bc"])).float().view(-1)
        f = torch.empty(n, fc.out_features, dtype=torch.bfloat16, device=y.device)
        v = value_out if value_out is not None else torch.empty(n, dtype=torch.float32,
                                                                 device=y.device)
        N.check(N.kernels().mbk_fc_fwd(y.data_ptr(), 1, self._fc_cache["w5"].data_ptr(),
                                       fc.bias.data_ptr(), self.critic.weight.data_ptr(),
                                       self.critic.bias.data_ptr(), n, I, fc.out_features,
                                       f.data_ptr(), v.data_ptr(), N.stream_ptr()), "fc_fwd")
        return f, v

    def _trunk(self, obs: torch.Tensor) -> torch.Tensor:
        """HIP conv trunk (NHWC bf16 [n, ho, wo, c], before the reference's Flatten/ReLU)."""
        if self._hip_enc is None or self._hip_enc.packed_fwd.device != obs.device:
            self._hip_enc = HipEncoder(self.h, self.w, self.planes, self.channels, obs.device)
        # fp8 MFMA convs for no-grad (acting) forwards when enabled (config 5);
        # gradient-carrying forwards always run the bf16 kernels
        self._hip_enc.fp8 = self.fp8_inference
        n = obs.shape[0] if obs.dim() == 2 else obs.numel() // (self.h * self.w)
        grad = torch.is_grad_enabled()
        pre = self._prepacked and not grad
        return encode(obs.reshape(n, self.h * self.w), self._hip_enc,
                      encoder_params(self.network, len(self.channels)), grad, prepacked=pre)

    def features(self, obs: torch.Tensor) -> torch.Tensor:
        if self._use_hip(obs):
            # conv trunk on the HIP MFMA kernels (NHWC bf16), then the reference's
            # NCHW flatten order into network.5
            y = self._trunk(obs)
            n = y.shape[0]
            pre = self._prepacked and not torch.is_grad_enabled()
            # ReLU -> network.5 -> ReLU on the NHWC rows: the Linear's input columns are
            # permuted from the reference's NCHW flatten order instead of the activations
            nseq = len(self.channels)
            _, ho, wo, c = y.shape
            f = F.relu(y.reshape(n, -1))
            f = linear(f, self.network[nseq + 2], nhwc=(c, ho, wo),
                       cached=(self._fc_cache["w5"],
                               self._fc_cache.get("b5", self.network[nseq + 2].bias.detach()))
                       if pre else None)
            return F.relu(f)
        x = self._planes(obs)
        with self._autocast(x):
            return self.network(x)

    def policy_value(self, obs: torch.Tensor):
        """(dense logits [N, 78*h*w], value [N]). On the HIP path both heads run on the
        hand-written MFMA GEMM (gemm.hip), never on hipBLASLt."""
        f = self.features(obs)
        if self._use_hip(obs):
            return linear(f, self.actor), linear(f, self.critic).float().view(-1)
        with self._autocast(f):
            logits = self.actor(f)
            value = self.critic(f)
        return logits, value.float().view(-1)

    def initial_state(self, batch_size: int = 1):
        """No recurrent state (reference model.py:139-141)."""
        return tuple()

    # ------------------------------------------------------------ acting / learning
    @torch.no_grad()
    def pack_inference(self, device) -> None:
        """Refresh every derived inference buffer from the fp32 parameters: packed conv
        weights (bf16 or fp8), the sparse head's packed blocks and bf16 FC/critic weights.
        After the first call, no-grad forwards skip all per-call packing (the acting graph
        is then only compute; the GPU engine replays a captured pack graph after each
        weight publish). Only for an inference copy whose weights change through publish."""
        dev = torch.device(device)
        if self._hip_enc is None or self._hip_enc.packed_fwd.device != dev:
            self._hip_enc = HipEncoder(self.h, self.w, self.planes, self.channels, dev)
        enc = self._hip_enc
        enc.fp8 = self.fp8_inference
        ws = [p.detach() for p in encoder_params(self.network, len(self.channels))[0::2]]
        if enc.fp8:
            enc.pack_fp8(ws)
        else:
            enc.pack(ws, with_bwd=False)
        self._head(dev).pack(self.actor.weight, self.actor.bias, with_t=False)
        nseq = len(self.channels)
        fc = self.network[nseq + 2]
        if fc.out_features == 256:
            # the fused trunk head (trunk.hip) reads fp32 b5 / wc / bc itself: only W5's
            # NHWC bf16 operand is derived, by one index-map gather (no ATen copies)
            key = (fc.out_features, enc.out_c) + tuple(enc.out_hw)
            if (self._tail_maps is None or self._tail_maps.key != key
                    or self._tail_maps.device != dev):
                self._tail_maps = TailMaps(*key, dev)
            if self._fc_cache is None or "w5" not in self._fc_cache:
                self._fc_cache = {"w5": torch.empty(self._tail_maps.fwd.shape,
                                                    dtype=torch.bfloat16, device=dev)}
            map_gather([(fc.weight.detach(), self._fc_cache["w5"], self._tail_maps.fwd)])
            self._prepacked = True
            return
        w5 = nhwc_weight(fc.weight.detach(), (enc.out_c,) + tuple(enc.out_hw))
        if self._fc_cache is None or "b5" not in self._fc_cache:
            self._fc_cache = {"w5": torch.empty(w5.shape, dtype=torch.bfloat16, device=dev),
                              "b5": torch.empty(fc.bias.shape, dtype=torch.bfloat16, device=dev),
                              "wc": torch.empty(self.critic.weight.shape, dtype=torch.bfloat16,
                                                device=dev),
                              "bc": torch.empty(self.critic.bias.shape, dtype=torch.bfloat16,
                                                device=dev)}
        c = self._fc_cache
        c["w5"].copy_(w5)
        c["b5"].copy_(fc.bias.detach())
        c["wc"].copy_(self.critic.weight.detach())
        c["bc"].copy_(self.critic.bias.detach())
        self._prepacked = True

    def _head(self, dev) -> SparseHead:
        if self._hip_head is None or self._hip_head.device != dev:
            self._hip_head = SparseHead(self.h * self.w, dev)
        return self._hip_head

    @torch.no_grad()
    def act(self, obs, mask_bits, rng_state=None, generator=None, action_out=None,
            logp_out=None, bucketed: bool = False, logits_out=None, value_out=None,
            act16_out=None):
        """Sample under the mask. Returns (action [N,S,7] u8, logp [N], value [N]).
        bucketed: the head's active pairs were bucketed by mbk_decode_obs_mask_bucket.
        logits_out: also write the dense policy logits [N, 78*h*w] (reference 'policy_logits';
        one extra dense head GEMM on gemm.hip, the sparse sampler does not need them)."""
        if self._use_hip(obs):
            # sparse head: only cells with a legal action are computed (ops/head.py)
            pre = self._prepacked
            if pre:
                self._hip_enc.fp8 = self.fp8_inference
                f, value = self._act_features(obs, value_out=value_out)
            else:
                f = self.features(obs)
                value = linear(f, self.critic).float().view(-1)
            n = f.shape[0]
            if logits_out is not None:
                logits_out.copy_(linear(f.to(torch.bfloat16), self.actor).float())
            action, logp = sparse_sample(f.to(torch.bfloat16), self.actor.weight, self.actor.bias,
                                         mask_bits.reshape(n, -1, 3), rng_state,
                                         self._head(f.device), action_out, logp_out,
                                         prepacked=pre, bucketed=bucketed, act16_out=act16_out)
            return action, logp, value
        logits, value = self.policy_value(obs)
        if logits_out is not None:
            logits_out.copy_(logits.float())
        action, logp = cell_head.sample(logits, mask_bits, rng_state, generator)
        return action, logp, value

    def evaluate(self, obs, mask_bits, action, n_score: int | None = None, abits=None):
        """Log-prob/entropy of ``action`` (first ``n_score`` rows) and values (all rows).

        Used by the learner on a time-major (T+1)*B batch: values are needed on
        all T+1 rows (bootstrap), the head only on the first T*B. abits: the scored rows'
        active-cell bitmap [n_score, S/32] from the acting step (HIP learner path only).
        """
        if self._use_hip(obs) and torch.is_grad_enabled():
            # learner: trunk, then ONE autograd node for network.5 + head + critic whose
            # backward kernels write every gradient (ops/tail.py). The head's compaction (and
            # its one host sync) goes first: it reads only masks / bitmap rows.
            n = obs.shape[0]
            ns = n if n_score is None else n_score
            self._head(obs.device).prepare_scoring(mask_bits.reshape(ns, -1, 3), ns, abits)
            y = self._trunk(obs)
            _, ho, wo, c = y.shape
            fc = self.network[len(self.channels) + 2]
            key = (fc.out_features, c, ho, wo)
            if (self._tail_maps is None or self._tail_maps.key != key
                    or self._tail_maps.device != y.device):
                self._tail_maps = TailMaps(*key, y.device)
            return impala_tail(y, fc, self.critic, self.actor, mask_bits.reshape(ns, -1, 3),
                               action.reshape(ns, -1, 7), ns, self._head(y.device),
                               self._tail_maps, abits)
        f = self.features(obs)
        if self._use_hip(obs):
            value = linear(f, self.critic).float().view(-1)
        else:
            with self._autocast(f):
                value = self.critic(f).float().view(-1)
        fh = f if n_score is None else f[:n_score]
        if self._use_hip(obs):
            logp, ent = sparse_score(fh.to(torch.bfloat16), self.actor.weight, self.actor.bias,
                                     mask_bits.reshape(fh.shape[0], -1, 3),
                                     action.reshape(fh.shape[0], -1, 7), self._head(f.device))
            return logp, ent, value
        with self._autocast(fh):
            logits = self.actor(fh)
        logp, ent = cell_head.score(logits, mask_bits, action)
        return logp, ent, value

    def get_action(self, input_dict: dict, learning: bool = False, inds=(), agent_state=()):
        """Reference-compatible API (model.py:165-216) on reference-layout inputs.

        input_dict["obs"]: (1,1,n,h,w,27) when acting, (N,h,w,27) when learning;
        ["action_mask"]: (1,n,78hw) / (N,78hw); ["action"] (N,7hw) when learning.
        Returns ({action, policy_logits, logprobs, baseline[, entropy]}, ()).
        On the GPU the one-hot obs are packed to bit planes and the whole call runs on the
        HIP kernels: conv trunk, gemm.hip for the dense actor logits (the reference output
        includes them), masked_cell.hip for the per-cell masked categoricals.
        """
        obs = input_dict["obs"]
        mask = input_dict["action_mask"]
        if not learning:
            obs = obs.reshape(-1, self.h, self.w, self.planes)
            mask = mask.reshape(obs.shape[0], -1)
        n = obs.shape[0]
        S = self.h * self.w
        maskb = mask.reshape(n, S, cell_head.CELL).bool()
        obs = self._compact_obs(obs)
        logits, value = self.policy_value(obs)
        if self._use_hip(obs):
            mbits = cell_head.pack_mask(maskb)
            lg = logits.float()
            if learning:
                a = input_dict["action"].reshape(n, S, cell_head.COMPS).to(torch.uint8)
                logp, ent = cell_head.score(lg, mbits, a)
                out = dict(action=a.view(n, -1).long(), policy_logits=lg, logprobs=logp,
                           baseline=value.view(1, -1), entropy=ent)
            else:
                with torch.no_grad():
                    act, logp = cell_head.sample(lg, mbits, self._rng(lg.device))
                out = dict(action=act.view(n, -1).long(), policy_logits=lg, logprobs=logp,
                           baseline=value.view(1, -1))
            return out, ()
        if learning:
            a = input_dict["action"].reshape(n, S, cell_head.COMPS)
            act, logp, ent = cell_head.cell_head_torch(logits.float(), maskb, a)
            out = dict(action=act.view(n, -1).long(), policy_logits=logits.float(), logprobs=logp,
                       baseline=value.view(1, -1), entropy=ent)
        else:
            with torch.no_grad():
                act, logp, _ = cell_head.cell_head_torch(logits.float(), maskb, None)
            out = dict(action=act.view(n, -1).long(), policy_logits=logits.float(),
                       logprobs=logp, baseline=value.view(1, -1))
        return out, ()

    def get_value(self, input_dict: dict, agent_state=(), learning=False, inds=()):
        obs = input_dict["obs"]
        if not learning:
            obs = obs.reshape(-1, self.h, self.w, self.planes)
        return self.policy_value(self._compact_obs(obs))[1].view(-1, 1)


def num_params(model: nn.Module) -> int:
    return int(sum(p.numel() for p in model.parameters()))


def reference_param_count(h: int, w: int) -> int:
    """Closed form used by tests (matches SURVEY §7.6 counts)."""
    m = Agent((h, w, 27))
    return num_params(m)


__all__ = ["Agent", "ConvSequence", "ResidualBlock", "layer_init", "num_params"]
