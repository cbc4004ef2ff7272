"""Bridge from compiled forward/backward traces to ``torch.autograd`` (parity: reference
``thunder/executors/torch_autograd.py:17-185``).

``ThunderFunction`` runs the compiled augmented forward; its backward calls the
compiled backward with a *list* of saved tensors + cotangents that the generated
program clears immediately, so activations are freed as the backward proceeds.
"""
from __future__ import annotations

import torch
from torch.autograd.function import once_differentiable


from ..core.pytree import LEAF as _LEAF

_ONE_TENSOR = [True]


class ThunderFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, entry, n_inputs, *flat_inputs):
        out, saved_tensors, saved_other = entry.forward_fn(*flat_inputs)
        if type(out) is torch.Tensor and entry.diff_output_mask == [True]:
            # the common case (a loss / one activation): no output tree to walk
            ctx.entry = entry
            ctx.overlap_params = getattr(entry, "_overlap_params", None)
            ctx.saved = list(saved_tensors) + list(saved_other)
            ctx.n_inputs = n_inputs
            ctx.out_is_tensor = _ONE_TENSOR
            ctx.diff_shapes = [tuple(out.shape)]
            entry._last_out_spec = _LEAF
            entry._last_flat_out = [out]
            ctx.set_materialize_grads(False)
            return (out,)
        from ..core.pytree import tree_flatten

        flat_out, out_spec = tree_flatten(out)
        ctx.entry = entry
        ctx.overlap_params = getattr(entry, "_overlap_params", None)
        ctx.saved = list(saved_tensors) + list(saved_other)
        ctx.n_inputs = n_inputs
        tensor_outs = []
        nondiff = []
        for o, diff in zip(flat_out, entry.diff_output_mask):
            if isinstance(o, torch.Tensor):
                tensor_outs.append(o)
                if not diff:
                    nondiff.append(o)
        ctx.out_is_tensor = [isinstance(o, torch.Tensor) for o in flat_out]
        # this call's differentiable output shapes (a symbolic-shape program serves many sizes; the
        # traced metadata holds only the first): zeros for missing cotangents take these
        ctx.diff_shapes = [tuple(o.shape) if isinstance(o, torch.Tensor) else None
                           for o, d in zip(flat_out, entry.diff_output_mask) if d]
        entry._last_out_spec = out_spec
        entry._last_flat_out = flat_out
        if nondiff:
            ctx.mark_non_differentiable(*nondiff)
        ctx.set_materialize_grads(False)
        return tuple(tensor_outs)

    @staticmethod
    @once_differentiable
    def backward(ctx, *grads):
        entry = ctx.entry
        args = ctx.saved
        keep = False
        try:  # backward(retain_graph=True): the saved tensors must survive this pass
            keep = torch._C._autograd._get_current_graph_task_keep_graph()
        except (AttributeError, RuntimeError):
            pass
        if args is None:
            raise RuntimeError("Trying to backward through the graph a second time (or directly access saved tensors "
                               "after they have already been freed); specify retain_graph=True on the first backward")
        if keep:
            args = list(args)  # the backward program clears the list it is handed
        else:
            ctx.saved = None
        # align tensor-output grads with the differentiable outputs
        gi = iter(grads)
        cts = []
        k = 0
        for is_t, diff in zip(ctx.out_is_tensor, entry.diff_output_mask):
            g = next(gi) if is_t else None
            if diff:
                cts.append(g)
        outs_meta = entry.diff_output_meta
        for i, g in enumerate(cts):
            if g is None:
                shape, dtype, device = outs_meta[i]
                if ctx.diff_shapes[i] is not None:
                    shape = ctx.diff_shapes[i]
                cts[i] = torch.zeros(shape, dtype=dtype, device=device)
        args.extend(cts)
        handled: set = set()
        if ctx.overlap_params:
            # the optimizer updates these parameters inside the backward (optimizer_overlap.py)
            from ..transforms.optimizer_overlap import active

            with active(entry.overlap_optimizer, ctx.overlap_params, handled):
                in_grads = entry.backward_fn(args)
        else:
            in_grads = entry.backward_fn(args)
        result = [None] * ctx.n_inputs
        for k, (idx, g) in enumerate(zip(entry.grad_input_indices, in_grads)):
            result[idx] = None if k in handled else g
        return (None, None, *result)


def connect_to_autograd(entry, flat_inputs):
    entry._overlap_params = None
    opt = entry.overlap_optimizer
    if opt is not None:
        # backward output k -> the parameter tensor the attached optimizer updates in the backward
        entry._overlap_params = {k: flat_inputs[i] for k, i in enumerate(entry.grad_input_indices)
                                 if opt.manages(flat_inputs[i])} or None
    outs = ThunderFunction.apply(entry, len(flat_inputs), *flat_inputs)
    entry._overlap_params = None
    from ..core.pytree import tree_unflatten

    if entry._last_out_spec is _LEAF:
        entry._last_flat_out = None
        return outs[0]
    flat_out = list(entry._last_flat_out)
    it = iter(outs)
    for i, o in enumerate(flat_out):
        if isinstance(o, torch.Tensor):
            flat_out[i] = next(it)
    entry._last_flat_out = None
    return tree_unflatten(flat_out, entry._last_out_spec)
