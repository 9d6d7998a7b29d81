"""Generate the golden fixtures under tests/golden/ from the reference's shipped data.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py

Everything here is DATA taken from files the reference ships; no reference
source is copied and nothing in a reference file is executed:

* graphs/graph-0.pt -- ``torch.load(weights_only=True)`` refuses it (it pickles
  a torch_geometric ``Data`` subclass).  We do NOT unpickle it.  A ``.pt`` file
  is a zip archive whose tensor storages are raw little-endian byte blobs
  (``graph-0/data/<k>``); we read those bytes with ``zipfile`` +
  ``numpy.frombuffer`` and identify each blob by its size (int64 [2,24000]
  edge_index; float32 [2000,10] x_s, [12,10] x_t, [24000,10] x_e, [1,10] u).
  -> graph0.npz
* params/model_gnn_0.pth and models/model_gnn_0.pth -- loaded with
  ``torch.load(weights_only=True)`` (accepted).  -> ckpt_params.npz,
  ckpt_models.npz (model state only).
* params/model_gnn_0.pth's ``optim_state`` (train.py:154-165 saves
  ``optimizer.state_dict()`` of torch.optim.Adam beside the model): the Adam
  step count, the indices of the parameters that have state (the ones the
  reference's backward ever gave a gradient) and their ``exp_avg`` /
  ``exp_avg_sq``, plus the param group's hyper-parameters.  -> ckpt_adam.npz
* params/*.txt -- class tables (T_i hours per visit, N_i galaxies).  -> classes.npz
"""
import os
import sys
import zipfile

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def graph0():
    z = zipfile.ZipFile(os.path.join(REF, "graphs/graph-0.pt"))
    blobs = {n: z.read(n) for n in z.namelist() if "/data/" in n and not n.endswith("serialization_id")}
    by_size = {len(b): b for b in blobs.values()}
    ei = np.frombuffer(by_size[2 * 24000 * 8], dtype="<i8").reshape(2, 24000)
    x_s = np.frombuffer(by_size[2000 * 10 * 4], dtype="<f4").reshape(2000, 10)
    x_t = np.frombuffer(by_size[12 * 10 * 4], dtype="<f4").reshape(12, 10)
    x_e = np.frombuffer(by_size[24000 * 10 * 4], dtype="<f4").reshape(24000, 10)
    u = np.frombuffer(by_size[10 * 4], dtype="<f4").reshape(1, 10)
    assert ei.min() >= 0 and ei[0].max() < 2000 and ei[1].max() < 12
    np.savez_compressed(
        os.path.join(HERE, "graph0.npz"),
        edge_index=ei.astype(np.int16), x_t=x_t,
        x_s_shape=np.array(x_s.shape), x_s_absmax=np.float32(np.abs(x_s).max()),
        x_e_shape=np.array(x_e.shape), x_e_absmax=np.float32(np.abs(x_e).max()),
        u_shape=np.array(u.shape), u_absmax=np.float32(np.abs(u).max()))


def checkpoints():
    import torch
    ck = torch.load(os.path.join(REF, "params/model_gnn_0.pth"), weights_only=True, map_location="cpu")
    arrs = {k: v.numpy() for k, v in ck["model_state"].items()}
    np.savez_compressed(os.path.join(HERE, "ckpt_params.npz"), epoch=np.int64(ck["epoch"]), **arrs)
    st = ck["optim_state"]["state"]
    grp = ck["optim_state"]["param_groups"][0]
    idx = sorted(st.keys())
    adam = {"indices": np.array(idx, dtype=np.int64),
            "step": np.array([float(st[i]["step"]) for i in idx]),
            "n_params": np.int64(len(grp["params"])), "lr": np.float64(grp["lr"]),
            "betas": np.array(grp["betas"], dtype=np.float64), "eps": np.float64(grp["eps"]),
            "weight_decay": np.float64(grp["weight_decay"])}
    for i in idx:
        adam[f"exp_avg_{i}"] = st[i]["exp_avg"].numpy()
        adam[f"exp_avg_sq_{i}"] = st[i]["exp_avg_sq"].numpy()
    np.savez_compressed(os.path.join(HERE, "ckpt_adam.npz"), **adam)
    sd = torch.load(os.path.join(REF, "models/model_gnn_0.pth"), weights_only=True, map_location="cpu")
    np.savez_compressed(os.path.join(HERE, "ckpt_models.npz"), **{k: v.numpy() for k, v in sd.items()})


def classes():
    out = {}
    for name in ["increasing", "decreasing", "classes", "small", "doubled"]:
        out[name] = np.loadtxt(os.path.join(REF, "params", name + ".txt")).astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "classes.npz"), **out)


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("reference not mounted; fixtures are already committed")
    graph0()
    checkpoints()
    classes()
    print("golden fixtures written to", HERE)
