"""Execution-free reader for the reference's precomputed cache
(``spirals.pkl`` / ``transforms.pkl`` / ``norm.pt``), so a reference
``precomputed_path`` drops in unchanged under ``manager.ModelManager``.

The reference caches its geometry precompute with plain ``pickle.dump``
(``model_manager.py:203-205, 227-228``).  Those files are untrusted data, so we
never hand them to ``pickle.load``.  Instead this module walks the opcode
stream with :func:`pickletools.genops` and builds values on a private stack.
Global references are kept as inert ``(module, name)`` markers; nothing named
by the file is imported or called.  Only three reconstructors are interpreted,
each re-implemented here:

* ``torch.storage._load_from_bytes(blob)`` -> the blob is a legacy
  ``torch.save`` of one storage; it is decoded with
  ``torch.load(..., weights_only=True)`` (torch's restricted unpickler).
* ``torch._utils._rebuild_tensor_v2(storage, offset, size, stride, ...)`` ->
  ``torch.as_strided`` view on that storage.
* ``torch._utils._rebuild_sparse_tensor(layout, (indices, values, size))`` ->
  ``{"indices", "values", "size"}`` dict (COO kept in file order).
* any other class marker + ``NEWOBJ``/``BUILD`` -> plain dict of its state
  (used for ``torch_geometric.data.data.Data``).
"""
import io
import pickletools

import torch


class _Global:
    def __init__(self, module, name):
        self.module, self.name = module, name

    def __repr__(self):
        return f"<global {self.module}.{self.name}>"


class _Obj(dict):
    """State of an object whose class is only known by name."""

    def __init__(self, cls):
        super().__init__()
        self.cls = cls


_MARK = object()


def _call(fn, args):
    if not isinstance(fn, _Global):
        raise ValueError(f"REDUCE on non-global {fn!r}")
    key = (fn.module, fn.name)
    if key == ("torch.storage", "_load_from_bytes"):
        (blob,) = args
        return torch.load(io.BytesIO(blob), weights_only=True)
    if key == ("torch._utils", "_rebuild_tensor_v2"):
        storage, offset, size, stride = args[:4]
        dtype = storage.dtype
        raw = storage._untyped_storage if hasattr(storage, "_untyped_storage") \
            else storage
        t = torch.empty(0, dtype=dtype)
        t.set_(raw, offset, tuple(size), tuple(stride))
        return t.clone()
    if key == ("torch._utils", "_rebuild_sparse_tensor"):
        layout, data = args
        indices, values, size = data[:3]
        return {"indices": indices, "values": values, "size": tuple(size)}
    if key == ("torch.serialization", "_get_layout"):
        return str(args[0])
    if key == ("collections", "OrderedDict"):
        return dict()
    if key == ("torch", "Size"):
        return tuple(args[0]) if args else tuple()
    if key == ("builtins", "getattr") and isinstance(args[0], _Global):
        return _Global(args[0].module, args[0].name + "." + args[1])
    raise ValueError(f"refusing to interpret {fn!r}")


def load(path):
    data = open(path, "rb").read()
    stack, memo = [], {}

    def pop_mark():
        items = []
        while True:
            x = stack.pop()
            if x is _MARK:
                break
            items.append(x)
        items.reverse()
        return items

    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        elif n == "STOP":
            return stack.pop()
        elif n == "MARK":
            stack.append(_MARK)
        elif n in ("EMPTY_LIST",):
            stack.append([])
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n in ("MEMOIZE",):
            memo[len(memo)] = stack[-1]
        elif n in ("BINPUT", "LONG_BINPUT"):
            memo[arg] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8",
                   "SHORT_BINBYTES", "BINBYTES", "BINBYTES8",
                   "BININT", "BININT1", "BININT2", "LONG1", "BINFLOAT"):
            stack.append(arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "TUPLE1":
            stack.append((stack.pop(),))
        elif n == "TUPLE2":
            b = stack.pop(); a = stack.pop(); stack.append((a, b))
        elif n == "TUPLE3":
            c = stack.pop(); b = stack.pop(); a = stack.pop()
            stack.append((a, b, c))
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n == "LIST":
            stack.append(pop_mark())
        elif n == "APPEND":
            v = stack.pop(); stack[-1].append(v)
        elif n == "APPENDS":
            items = pop_mark(); stack[-1].extend(items)
        elif n == "SETITEM":
            v = stack.pop(); k = stack.pop(); stack[-1][k] = v
        elif n == "SETITEMS":
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif n == "STACK_GLOBAL":
            name = stack.pop(); module = stack.pop()
            stack.append(_Global(module, name))
        elif n == "GLOBAL":
            module, name = arg.split(" ")
            stack.append(_Global(module, name))
        elif n == "REDUCE":
            args = stack.pop(); fn = stack.pop()
            stack.append(_call(fn, args))
        elif n == "NEWOBJ":
            args = stack.pop(); cls = stack.pop()
            stack.append(_Obj(cls))
        elif n == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(state, tuple) and len(state) == 2:
                st, slots = state
                for part in (st, slots):
                    if isinstance(part, dict):
                        obj.update(part)
            elif isinstance(state, dict):
                obj.update(state)
            else:
                raise ValueError("unsupported BUILD state")
        else:
            raise ValueError(f"unsupported pickle opcode {n}")
    raise ValueError("no STOP opcode")


def load_precomputed(path):
    """The reference's ``precomputed_path`` (model_manager.py:176-230) as a
    dict in the ``topology_craniofacial.npz`` layout (spirals, down/up COO in
    file order, low-resolution faces/positions), read without executing
    anything from the files.  The template itself (regions, Laplacian) is
    added by the caller."""
    import os

    import numpy as np
    spirals = load(os.path.join(path, "spirals.pkl"))
    low, down, up = load(os.path.join(path, "transforms.pkl"))
    if not (len(spirals) == len(down) == len(up) == len(low)):
        raise ValueError(f"{path}: spirals / transforms level counts differ")
    out = {"n_levels": np.int32(len(spirals))}
    for l in range(len(spirals)):
        out[f"spiral_{l}"] = spirals[l].numpy().astype(np.int32)
        for name, tr in (("down", down[l]), ("up", up[l])):
            idx = tr["indices"].numpy()
            out[f"{name}_{l}_row"] = idx[0].astype(np.int32)
            out[f"{name}_{l}_col"] = idx[1].astype(np.int32)
            out[f"{name}_{l}_val"] = tr["values"].numpy().astype(np.float32)
            out[f"{name}_{l}_shape"] = np.asarray(tr["size"], np.int64)
        out[f"pos_{l + 1}"] = low[l]["pos"].numpy().astype(np.float32)
        out[f"face_{l + 1}"] = low[l]["face"].numpy().T.astype(np.int32)
    return out
