"""Device-backed CoordinateTree — the reference's node API over HBM tensors.

Reference: CoordinateTree.py:4-36.  The reference allocates an object array of
S1 + S1^2 + S1^3 slots (CoordinateTree.py:5-9; 736 MB at S1 = 451) but
predictive_control only ever writes nodes 0..S1-1 of each layer
(math_model_tree.py:310-350, SURVEY Fact 1).  This class keeps the same flat
index space and parent arithmetic, but stores only the used nodes:

    states   float64 [n_layers, 3, S1]   (x, y, phi) per layer and node, in HBM
    controls float64 [2, S1]             (v, beta) of node k (same every layer)

Flat index j of layer l >= 1 is offset(l) + k with offset(l) = S1 + ... + S1^l;
layer 0 is j = k.  Slots the reference never writes read back as None, as an
unwritten slot of `np.empty(n, tuple)` does.  The kernel fills `states`
directly (mpc_rollout_argmin's states_out), so building the tree costs one
write of 24 B per node instead of a 91.9 M-slot allocation.
"""
import torch


class CoordinateTree:
    def __init__(self, size_max_1, n_layers=3, device=None):
        self.size_1 = int(size_max_1)
        self.size_2 = self.size_1 * self.size_1
        self.size_3 = self.size_2 * self.size_1
        self.n_layers = int(n_layers)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.offsets = [0]
        span = self.size_1
        for _ in range(1, self.n_layers):
            self.offsets.append(self.offsets[-1] + span)
            span *= self.size_1
        self._size = self.offsets[-1] + span if self.n_layers else 0
        self.states = torch.zeros((self.n_layers, 3, max(self.size_1, 1)), dtype=torch.float64,
                                  device=self.device)
        self.controls = torch.zeros((2, max(self.size_1, 1)), dtype=torch.float64,
                                    device=self.device)
        self.written = torch.zeros((self.n_layers, max(self.size_1, 1)), dtype=torch.bool)
        self._host = None

    # -- index arithmetic (CoordinateTree.py:20-30) -------------------------------
    def _locate(self, index):
        """flat index -> (layer, node) or (layer, None) for a slot never used."""
        if index < 0 or index >= self._size:
            raise IndexError(f"index {index} out of range for size {self._size}")
        layer = 0
        for l in range(self.n_layers - 1, -1, -1):
            if index >= self.offsets[l]:
                layer = l
                break
        k = index - self.offsets[layer]
        return layer, (k if k < self.size_1 else None)

    def _layer_of(self, j):
        """Layer by the reference's thresholds; like its final `else`, any
        j past the last layer's start counts as the last layer (no bounds)."""
        for l in range(self.n_layers - 1, 0, -1):
            if j >= self.offsets[l]:
                return l
        return 0

    def get_index_of_parent(self, index_of_element):
        """Layer 0: itself; layer 1: (j - S1) % S1; layer >= 2: [parent,
        grandparent, ...] down to layer 0 (for 3 layers: [S1 + k, k], as the
        reference's recursion returns).  Pure index arithmetic, no bounds
        check, as in CoordinateTree.py:20-30."""
        j = index_of_element
        layer = self._layer_of(j)
        if layer == 0:
            return j
        if layer == 1:
            return (j - self.size_1) % self.size_1
        chain = []
        while layer >= 1:
            j = self.offsets[layer - 1] + ((j - self.offsets[layer]) % self.size_1)
            chain.append(j)
            layer -= 1
        return chain

    def get_size(self):
        return self._size

    # -- node access ---------------------------------------------------------------
    def _materialise(self):
        if self._host is None:
            self._host = (self.states.cpu(), self.controls.cpu())
        return self._host

    def mark_filled(self):
        """Called after the kernel wrote `states`/`controls` for every node."""
        self.written[:] = True
        self._host = None

    def __getitem__(self, index):
        layer, k = self._locate(int(index))
        if k is None or not bool(self.written[layer, k]):
            return None
        st, ctl = self._materialise()
        return [float(st[layer, 0, k]), float(st[layer, 1, k]), float(st[layer, 2, k]),
                float(ctl[0, k]), float(ctl[1, k])]

    def __setitem__(self, index, coordinates):
        layer, k = self._locate(int(index))
        if k is None:
            raise IndexError(f"slot {index} is outside the used nodes of layer {layer}")
        vals = [float(c) for c in coordinates]
        self.states[layer, :, k] = torch.tensor(vals[:3], dtype=torch.float64)
        if len(vals) >= 5:
            self.controls[:, k] = torch.tensor(vals[3:5], dtype=torch.float64)
        self.written[layer, k] = True
        self._host = None

    def clear(self):
        self.states.zero_()
        self.controls.zero_()
        self.written[:] = False
        self._host = None

    def __str__(self):
        st, ctl = self._materialise()
        rows = []
        for layer in range(self.n_layers):
            for k in range(self.size_1):
                if bool(self.written[layer, k]):
                    rows.append(f"{self.offsets[layer] + k}: [{st[layer, 0, k]!r}, "
                                f"{st[layer, 1, k]!r}, {st[layer, 2, k]!r}, "
                                f"{ctl[0, k]!r}, {ctl[1, k]!r}]")
        return "CoordinateTree(S1=%d, layers=%d, size=%d)\n%s" % (
            self.size_1, self.n_layers, self._size, "\n".join(rows))
