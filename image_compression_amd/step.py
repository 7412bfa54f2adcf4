"""One training step of the hot path — forward, RD loss, backward and (for
N > 1 processes) the gradient all-reduce — replayed from a hipGraph.

The reference runs this step as eager PyTorch under `nn.DataParallel`
(engine/trainer.py:163-209, 256-259): every op is a separate host-side launch.
A C2 step here is ~170 HIP kernels, many of them on the 16x16..4x4 hyperprior
maps where a launch is worth more than the work, so the whole step is
captured once into a hipGraph (`torch.cuda.CUDAGraph`; our C-ABI kernels
launch on torch's current stream, which is the capture stream during capture)
and replayed: one host call per step, no inter-kernel launch gaps.

Graph-safety of the step:
* inputs: the batch is copied into a static device tensor (`x`);
* workspace: every op takes its scratch from the caching allocator, which
  serves a capture from the graph's private pool;
* training noise: Philox counters come from a device-resident {seed, base}
  advanced by a kernel at the top of each forward (noise.py), so every replay
  draws fresh noise;
* gradients: views into one flat fp32 buffer, zeroed inside the graph and
  accumulated in place by autograd — so for N > 1 the whole gradient is ONE
  contiguous RCCL all-reduce (40.6 MB at C2) after the replay.

`graph=False` runs the same step eagerly (debugging, parity).
"""
import torch
import torch.distributed as dist


class TrainStep:
    """flat=True: gradients are views of one flat buffer (zeroed and accumulated
    in place inside the step) so a multi-process run all-reduces them with one
    RCCL call; flat=False (single process): autograd allocates each gradient
    inside the step (no zeroing / accumulation kernels)."""

    def __init__(self, model, example_x, graph=True, warmup=3, flat=None):
        if not example_x.is_cuda:
            raise RuntimeError("TrainStep needs a ROCm device tensor")
        self.model = model
        self.params = [p for p in model.parameters() if p.requires_grad]
        dev = example_x.device
        if flat is None:
            flat = dist.is_initialized() and dist.get_world_size() > 1
        self.flat_grad = None
        if flat:
            numel = sum(p.numel() for p in self.params)
            self.flat_grad = torch.zeros(numel, device=dev, dtype=torch.float32)
            off = 0
            for p in self.params:
                p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
                off += p.numel()
        self.x = example_x.detach().clone()
        self.graph = None
        self.losses = None
        if graph:
            self._capture(warmup)

    def _step(self):
        if self.flat_grad is not None:
            self.flat_grad.zero_()
        else:
            for p in self.params:
                p.grad = None
        _, losses = self.model(self.x)
        losses["total_loss"].backward()
        return losses

    def _eager(self):
        losses = self._step()
        return {k: v.detach() for k, v in losses.items()}

    def _capture(self, warmup):
        side = torch.cuda.Stream(self.x.device)
        side.wait_stream(torch.cuda.current_stream(self.x.device))
        with torch.cuda.stream(side):
            for _ in range(warmup):       # allocator pools warm, kernels loaded
                self._eager()
        torch.cuda.current_stream(self.x.device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            losses = self._step()
        # keep the graph's static loss outputs, not the autograd graph behind them: that graph
        # holds the parameters' AccumulateGrad nodes made on the capture stream, and a later
        # eager step through those nodes would accumulate its gradients on the capture stream
        # (torch: "AccumulateGrad node's stream does not match") -- a cross-stream use the
        # caching allocator is not told about
        self.losses = {k: v.detach() for k, v in losses.items()}
        del losses

    def __call__(self, x=None):
        """Run one step; returns the loss dict (0-dim device tensors; with a
        graph these are the graph's static outputs, overwritten next step)."""
        if x is not None:
            self.x.copy_(x)
        if self.graph is not None:
            self.graph.replay()
            losses = self.losses
        else:
            losses = self._eager()
        if self.flat_grad is not None and dist.is_initialized() and dist.get_world_size() > 1:
            from .distributed import all_reduce_mean_
            all_reduce_mean_(self.flat_grad)
        return losses

    def grads(self):
        """Current gradients as one flat tensor (a copy when flat=False)."""
        if self.flat_grad is not None:
            return self.flat_grad
        return torch.cat([p.grad.reshape(-1) for p in self.params])
