"""Result / checkpoint I/O with the reference's entry points (jaxsrc/solver.py:13-33).

The reference pickles ``(results, errs_all)`` (final) and
``[max_iters, phi_all, rho_all, alp_all, errs_all]`` (middle results).  Pickle
executes code on load, so this module stores the same nested structure as a
``.npz`` of arrays plus a JSON description of the nesting, loadable with
``allow_pickle=False`` and without jax.
"""
import json
import os

import numpy as np


def _flatten(obj, arrays):
    if isinstance(obj, (list, tuple)):
        return {"t": "list" if isinstance(obj, list) else "tuple", "v": [_flatten(o, arrays) for o in obj]}
    if isinstance(obj, (int, float, np.integer, np.floating)) and not isinstance(obj, bool):
        return {"t": "scalar", "v": float(obj) if isinstance(obj, (float, np.floating)) else int(obj)}
    arr = np.asarray(obj)
    key = "a{}".format(len(arrays))
    arrays[key] = arr
    return {"t": "array", "k": key}


def _unflatten(node, arrays):
    t = node["t"]
    if t == "list":
        return [_unflatten(n, arrays) for n in node["v"]]
    if t == "tuple":
        return tuple(_unflatten(n, arrays) for n in node["v"])
    if t == "scalar":
        return node["v"]
    return arrays[node["k"]]


def save(save_dir, filename, results):
    """solver.py:13-19 — writes <save_dir>/<filename>.npz."""
    os.makedirs(save_dir, exist_ok=True)
    arrays = {}
    tree = _flatten(results, arrays)
    path = os.path.join(save_dir, "{}.npz".format(filename))
    np.savez(path, __tree__=np.frombuffer(json.dumps(tree).encode(), dtype=np.uint8), **arrays)
    return path


def _load(path):
    with np.load(path, allow_pickle=False) as z:
        tree = json.loads(bytes(z["__tree__"]).decode())
        arrays = {k: z[k] for k in z.files if k != "__tree__"}
    return _unflatten(tree, arrays)


def load_solution(dir, filename):
    """solver.py:21-26 — returns (results, errors)."""
    results, errors = _load(os.path.join(dir, "{}.npz".format(filename)))
    return results, errors


def load_middle_solution(dir, filename):
    """solver.py:28-33 — returns [max_iters, phi_all, rho_all, alp_all, errs_all] (+ [phi_end, stepsz_param]
    when written by pdhg_amd.utils_pdhg_solver.PDHG_multi_step, which needs them to resume)."""
    return _load(os.path.join(dir, "{}.npz".format(filename)))
