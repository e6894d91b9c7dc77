"""Layer-split pipeline over ranks (LLaMA-65B across 1/2/4/8 GPUs).

One process per GPU.  Stage s of S owns the contiguous layers
[s*L/S, (s+1)*L/S) of the model file (weights + its KV-cache slice); stage 0
also owns tok_embeddings, stage S-1 the final norm and lm_head.  Per
llama_eval the residual stream `inpL` (f32 [N x n_embd], 32 KiB per decode
token at 65B) goes from stage s to s+1 with a point-to-point send/recv --
torch.distributed over RCCL (backend "nccl": the buffer stays in HBM and moves
over xGMI) or gloo (host buffer; CPU tests and single-GPU rehearsal).  The
last stage's greedy token is broadcast so stage 0 can embed it.

This replaces running llama_eval_internal (llama.cpp:927-1197) in one
process; nothing is reduced across ranks -- the only exchange is the
stage-to-stage hand-off (no all-reduce, no TP).
"""
import numpy as np


def layer_ranges(n_layer, n_stages):
    """contiguous split: stage s owns [s*L/S, (s+1)*L/S)"""
    if n_stages < 1 or n_stages > n_layer:
        raise ValueError("need 1 <= stages <= n_layer")
    return [(s * n_layer // n_stages, (s + 1) * n_layer // n_stages) for s in range(n_stages)]


class StagePipeline:
    """Drive one pipeline stage.  `stage` is an lvk.Llama created with
    layers=(begin, end) (or any object with the same stage_eval/get_x/set_x/
    logits methods); `dist` is torch.distributed, already initialised."""

    def __init__(self, stage, n_embd, n_ctx, dist, on_device, device=None, group=None):
        import torch
        self.torch = torch
        self.stage = stage
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.n_embd = n_embd
        self.on_device = on_device
        dev = device if on_device else "cpu"
        self.buf = torch.empty(n_ctx * n_embd, dtype=torch.float32, device=dev)
        self.tok = torch.zeros(1, dtype=torch.int64, device=dev)

    @property
    def first(self):
        return self.rank == 0

    @property
    def last(self):
        return self.rank == self.world - 1

    def _ptr(self, n):
        return self.buf.data_ptr(), n

    def eval(self, tokens, n_past):
        """all ranks call with the same tokens (only stage 0 reads them); returns
        the logits on the last stage, None elsewhere"""
        n = len(tokens)
        seg = self.buf[: n * self.n_embd]
        if not self.first:
            self.dist.recv(seg, src=self.rank - 1, group=self.group)
            if self.on_device:
                self.torch.cuda.synchronize()
            self.stage.set_x(seg.data_ptr(), n, self.on_device)
            self.stage.stage_eval(None, n, n_past)
        else:
            self.stage.stage_eval(np.asarray(tokens, np.int32), n, n_past)
        if not self.last:
            self.stage.get_x(seg.data_ptr(), n, self.on_device)
            self.dist.send(seg, dst=self.rank + 1, group=self.group)
            return None
        return self.stage.logits()

    def greedy_next(self, logits):
        """argmax on the last stage, broadcast to every stage"""
        if self.last:
            self.tok.fill_(int(np.argmax(logits[-1])))
        elif self.on_device:
            self.torch.cuda.synchronize()
        self.dist.broadcast(self.tok, src=self.world - 1, group=self.group)
        return int(self.tok.item())

    def decode(self, prompt, n_steps, n_past=0):
        """prompt then n_steps greedy tokens; returns the generated ids (all ranks)"""
        lg = self.eval(prompt, n_past)
        n_past += len(prompt)
        out = []
        tok = self.greedy_next(lg)
        for _ in range(n_steps):
            out.append(tok)
            lg = self.eval([tok], n_past)
            n_past += 1
            tok = self.greedy_next(lg)
        return out
