"""CPU stand-in for one rank's engine in the distributed PTMA warm-start chain protocol (TEST INFRASTRUCTURE ONLY).

It implements the staged-launch calls is3d2_amd.dist.launch_chained makes on an engine (launch_begin, chain_passes,
chain_pass, chain_end, launch_end, chain_boundary_size / _get / _put) with the oracle's chain step
(oracle.FamodChain, MomentumSpectra.cpp:1288-1368) as the worker, so the gloo tests run the protocol itself -- the
same code bench.py drives over RCCL -- on the CPU.  It follows engine.hip's k_chain_pass / k_chain_finish at the
granularity of one segment per chain and rank:

  pass 0      every chain's positions [q0, q1) from a cold start (exact on rank 0);
  pass j > 0  a chain whose incoming state (the predecessor's pass j - 1 end state) differs bitwise from the start of
              its stored run is walked again from the new start (cells past a re-synchronisation come out as stored);
  finisher    walks again from the predecessor's final state when this rank's last pass changed an end state or the
              predecessor walked, and passes its final states and walk flag on.

The boundary layout is the engine's: [f C + c] for state field f (prev_ok, lambda, aT, aL) of chain c, [4 C] = walk
flag (slot 2)."""
import numpy as np

from oracle import oracle as O


class EmuChainEngine:
    def __init__(self, spec, surf, q0, q1, npass=24):
        self.n = len(surf["tau"])
        self.C = max(1, min(int(spec["params"]["famod_chains"]), self.n))
        self.q0, self.q1, self.npass = q0, q1, npass
        self.walker = O.FamodChain(spec, surf)
        self.iters = None

    def _cells(self, c):
        return np.arange(c + self.q0 * self.C, min(self.n, self.q1 * self.C), self.C)

    def launch_begin(self, out_ptr=None, stream_ptr=None):
        C = self.C
        self.bin = np.zeros((3, 4 * C + 1))
        self.bout = np.zeros((3, 4 * C + 1))
        self.sstart = np.zeros((C, 4))
        self.end = np.zeros((C, 4))
        self.changed = [False] * self.npass
        self.iters = {c: None for c in range(C)}
        self.states = {c: None for c in range(C)}

    def chain_passes(self):
        return self.npass

    def chain_boundary_size(self):
        return 4 * self.C + 1

    def _walk(self, c, start):
        states, it, end = self.walker.walk(self._cells(c), start)
        self.states[c], self.iters[c] = states, it
        self.sstart[c] = start
        return end if len(it) else np.array(start, dtype=np.float64)

    def _start(self, slot, c):
        return self.bin[slot][[c, self.C + c, 2 * self.C + c, 3 * self.C + c]] if self.q0 > 0 else np.zeros(4)

    def _publish(self, slot):
        for c in range(self.C):
            for f in range(4):
                self.bout[slot][f * self.C + c] = self.end[c][f]

    def chain_pass(self, j):
        for c in range(self.C):
            if j == 0:
                self.end[c] = self._walk(c, np.zeros(4))
                self.changed[0] = self.q0 > 0        # cold starts: exact only without a predecessor
                continue
            st0 = self._start((j - 1) & 1, c)
            if st0.tobytes() == self.sstart[c].tobytes():
                continue
            new = self._walk(c, st0)
            if new.tobytes() != self.end[c].tobytes():
                self.changed[j] = True
            self.end[c] = new
        self._publish(j & 1)
        if j == 0:
            self._publish(1)

    def chain_end(self):
        walk = self.changed[self.npass - 1] or (self.q0 > 0 and self.bin[2][4 * self.C] != 0.0)
        if walk:
            for c in range(self.C):
                st0 = self._start(2, c)
                if st0.tobytes() != self.sstart[c].tobytes():
                    self.end[c] = self._walk(c, st0)
        self._publish(2)
        self.bout[2][4 * self.C] = 1.0 if walk else 0.0

    def launch_end(self):
        pass

    def chain_boundary_get(self, slot, buf):
        buf.numpy()[:] = self.bout[slot]

    def chain_boundary_put(self, slot, buf):
        self.bin[slot][:] = buf.numpy()

    def iterations(self):
        """Newton iterations of this range's stored solutions (the engine's k_chain_count)."""
        return int(sum(it[it > 0].sum() for it in self.iters.values() if it is not None))

    def final_states(self):
        """The chain state after every cell of the range, {cell: state}."""
        out = {}
        for c in range(self.C):
            for cell, st in zip(self._cells(c), self.states[c]):
                out[int(cell)] = st
        return out
