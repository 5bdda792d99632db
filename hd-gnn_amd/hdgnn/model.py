"""Drop-in for the reference's model_N.graph2graph, backed by libhdgnn.so.

graph2graph here is model_2 (HD-GNN/S, the reference main.py's import); hdgnn.model_1 /
model_3 / model_4 export the same class for the other variants (variant attribute).

Same constructor (model_2.py:16-33), same train(args) / test(args) flow, files and
printed lines (model_2.py:336-407, 434-548); the TF graph + sess.run are replaced by
the engine (hdgnn.engine.Engine -> C ABI -> k_commit_step on MI355X):

    reference                                         here
    sess.run([..., trainer], feed_dict) (369-383)     Engine.train_step(DeviceBatch)
    sess.run([loss, loss_map, C_edge_output2]) (486)  Engine.forward(DeviceBatch)
    read_data(self, Step) -> 12 dense arrays          reader(self, Step) -> the same tuple,
                                                      then data.compact_from_read_data
    saver.save / restore (427-451)                    TF V2 bundle, TF variable names

Reference behaviours kept on purpose: every batch feeds the maps
of the first Mini_batch commits (B.2, also in test); remainder commits are dropped
(B.3); test() looks for its checkpoint under checkpoint_dir/Repo/Repo/model_2/Step and
so normally evaluates freshly initialised weights (B.8).

Data parallel: when torch.distributed is initialised with world W > 1, every batch of
Mini_batch commits is split into W contiguous shards (Mini_batch % W == 0); the flat
gradient is all-reduced once per step (Engine.allreduce).  The epoch accuracy's correct
count is computed on the device and travels in the gradient trailer, so the same
all-reduce sums it.  Outputs written to disk are gathered on rank 0.
"""
import ctypes
import os
import time

import numpy as np

from . import _lib, layout, metrics, tfckpt
from .data import compact_from_read_data, onehot_relations

HS = 20   # De_e = De_er = h_size compiled into the engine
FAULT_POLL = 16   # train(): steps between fault polls inside a long epoch


def shard_plan(n_commits, mini_batch, world=1, rank=0):
    """Per reference batch j (floor division, model_2.py:364): this rank's commit range and
    the batch positions whose maps it feeds (Esc/Etc/..[:Mini_batch], model_2.py:376-381)
    -> list of ((commit_lo, commit_hi), (pos_lo, pos_hi))."""
    if mini_batch % world:
        raise ValueError("Mini_batch=%d is not divisible by world=%d" % (mini_batch, world))
    lb = mini_batch // world
    lo = rank * lb
    return [((j * mini_batch + lo, j * mini_batch + lo + lb), (lo, lo + lb))
            for j in range(n_commits // mini_batch)]


def _default_reader(model, step):
    """The reference's own loader (utils2.read_data), imported from the caller's path the
    way model_2.py does (`from utils2 import read_data`)."""
    try:
        from utils2 import read_data
    except ImportError as e:       # no silent fallback: the dataset loader is the caller's
        raise ImportError("graph2graph needs a reader: pass reader=... or put the reference's "
                          "utils2.py on sys.path") from e
    return read_data(model, step)


def _evaluation_funcs():
    """The reference's metrics module, imported from the caller's path the way model_2.py
    does (`from EvaluationFuncs import *`, model_2.py:12; the north star keeps it as-is);
    hdgnn.metrics (the same functions restated, pinned by the reference's own outputs in
    tests/golden/metrics_tiny.*) only when EvaluationFuncs is not importable."""
    try:
        import EvaluationFuncs
        return EvaluationFuncs
    except ImportError:
        return metrics


_COUNT_W = np.array([1, 1 << 16, 1 << 32], dtype=np.int64)   # trailer count parts


class Saver(object):
    """tf.train.Saver() of build_model (model_2.py:139): every variable of the graph
    (tf.global_variables() at that point: the model's weights) saved
    as a TF V2 bundle under the TF variable names (hdgnn.tfckpt), plus this engine's TF1
    Adam slots and beta powers so a restore resumes training.  save() keeps the newest
    max_to_keep bundles (TF's default 5) and rewrites the 'checkpoint' state file, as
    Saver.save does; restore() reads a TF-written bundle too (no Adam slots: the
    optimizer state is then left as it is).  The bundle bytes are assembled and written
    by libhdgnn (tfckpt.BundleTemplate -> hdg_bundle_write); background saves go to its
    native writer thread (tfckpt.BundleWriter), which also takes the training loop's
    result-file lines, so their file writes never run on the training thread."""

    def __init__(self, model, max_to_keep=5):
        self._model = model
        self.max_to_keep = max_to_keep
        self._last = []              # prefixes saved by this Saver, oldest first
        self._dropped = []           # prefixes whose removal is queued on the writer
        self._splits = {}            # prefix -> (directory, basename)
        self._tmpl = None
        self._writer = None
        self._dirs = set()           # directories known to exist

    def _template(self):
        if self._tmpl is None:
            self._tmpl = tfckpt.BundleTemplate(self._model.variant)
        return self._tmpl

    def writer(self):
        """The native background writer (created on first use)."""
        if self._writer is None:
            self._writer = tfckpt.BundleWriter(self._template())
        return self._writer

    def _host_state(self):
        """[params | adam_m | adam_v | beta_pow] (layout.state_offsets) in one device->host
        copy."""
        return self._model.engine.state.detach().cpu().numpy().copy()

    def _mkdir(self, d):
        if d not in self._dirs:
            os.makedirs(d, exist_ok=True)
            self._dirs.add(d)

    def _split(self, prefix):
        """(directory, basename) of a prefix, memoised (the training loop books one save
        per epoch against the same few prefixes)."""
        r = self._splits.get(prefix)
        if r is None:
            if len(self._splits) > 4096:
                self._splits.clear()
            d, base = os.path.split(prefix)
            r = self._splits[prefix] = (d or ".", base)
        return r

    def _book(self, prefix):
        """max_to_keep bookkeeping of a save at prefix: (paths to delete, state-file path,
        state-file text)."""
        d, base = self._split(prefix)
        if prefix in self._last:
            self._last.remove(prefix)
        self._last.append(prefix)
        removes = []
        while self.max_to_keep and len(self._last) > self.max_to_keep:
            old = self._last.pop(0)
            self._dropped.append(old)
            removes += [old + ".index", old + ".data-00000-of-00001"]
        kept = [b for dq, b in map(self._split, self._last) if dq == d]
        return removes, os.path.join(d, "checkpoint"), tfckpt.state_file_text(base, kept)

    def save(self, sess, save_path, global_step=None, background=False, state=None):
        """background=True: the writer thread writes the bundle of this state (a host copy
        taken now, so it holds exactly this step's values) while the caller's next steps
        run; flush() waits for it and raises its error.  state: a host copy of the flat
        training state the caller already holds (graph2graph.train reads it with the epoch's
        statistics), instead of a fresh device read."""
        prefix = save_path if global_step is None else "%s-%d" % (save_path, int(global_step))
        state = self._host_state() if state is None else state
        self._mkdir(self._split(prefix)[0])
        if not background:
            self.flush()
            return self._write(prefix, state)
        self._check(self.writer().poll)    # an earlier background save failed: raise now
        removes, spath, text = self._book(prefix)
        self.writer().submit(prefix, state, removes, spath, text)
        return prefix

    def flush(self):
        if self._writer is not None:
            self._check(self._writer.flush)
            self._dropped = []           # every queued removal has run

    def _check(self, op):
        """Run the writer's flush / poll; on a failed background job re-book the keep-list
        from the files on disk before raising: the failed prefix (no index file: bundles
        are written under .tmp and renamed) leaves it, and the older bundles that job
        would have removed (it stopped before its removals) come back, oldest first, so
        the next save's max_to_keep bookkeeping deletes them and no state file lists a
        bundle that was never written."""
        try:
            op()
        except tfckpt.CheckpointError:
            def there(q):
                return os.path.exists(q + ".index")
            back = [q for q in self._dropped if there(q) and q not in self._last]
            self._last = back + [q for q in self._last if there(q)]
            self._dropped = []
            raise

    def _write(self, prefix, state):
        self._template().write(prefix, state)
        removes, spath, text = self._book(prefix)
        for f in removes:
            if os.path.exists(f):
                os.remove(f)
        with open(spath, "w") as f:
            f.write(text)
        return prefix

    def restore(self, sess, save_path):
        import torch
        self.flush()
        eng = self._model.engine
        flat, m, v, bp = tfckpt.engine_state(tfckpt.read(save_path), self._model.variant)
        eng.set_params(flat)
        if m is not None:
            eng.m.copy_(torch.from_numpy(np.asarray(m, np.float32)))
            eng.v.copy_(torch.from_numpy(np.asarray(v, np.float32)))
            eng.beta_pow.copy_(torch.from_numpy(np.asarray(bp, np.float32)))


class graph2graph(object):
    variant = 2        # model_<variant>.py

    def __init__(self, sess, Ds, Ne, Nc, Ner, Ncr, Dr, De_e, De_er, Mini_batch, checkpoint_dir,
                 epoch, Ds_inter, Dr_inter, Step, Repo, *, reader=None, device=None, seed=0,
                 lr=3e-4, process_group=None, loader="utils2", data_root=".", compact=None):
        self.sess = sess                       # accepted and ignored (no TF session)
        self.Ds, self.Ne, self.Nc, self.Ner, self.Ncr, self.Dr = Ds, Ne, Nc, Ner, Ncr, Dr
        self.Ds_inter, self.Dr_inter = Ds_inter, Dr_inter
        self.De_e, self.De_er = De_e, De_er
        self.mini_batch_num = Mini_batch
        self.epoch = epoch
        self.checkpoint_dir = checkpoint_dir
        self.Step, self.Repo = Step, Repo
        self.reader = reader or _default_reader
        if loader not in ("utils2", "fast"):
            raise ValueError("loader must be 'utils2' (the reference read_data) or 'fast'")
        self.loader, self.data_root = loader, data_root
        # (train, test, maps) CommitBatches already in compact form (hdgnn.loader.read_compact,
        # a synthetic generator): used instead of reading the dataset
        self._given = compact
        self.seed, self.lr, self.pg = seed, lr, process_group
        self.device = device
        if (Ds, Dr, De_e, De_er) != (1, 2, HS, HS):
            raise ValueError("the engine is built for Ds=1, Dr=2, De_e=De_er=20 (got %s)"
                             % ((Ds, Dr, De_e, De_er),))
        if Ner != Ne * (Ne - 1) or Ncr != Nc * (Nc - 1):
            raise ValueError("Ner/Ncr must be Ne(Ne-1)/Nc(Nc-1) (complete relation digraphs)")
        self.build_model()

    # ------------------------------------------------------------------ model
    def build_model(self):
        import torch
        from .engine import Engine
        dist = torch.distributed
        self.world = dist.get_world_size(self.pg) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(self.pg) if self.world > 1 else 0
        if self.mini_batch_num % self.world:
            raise ValueError("Mini_batch=%d is not divisible by world=%d"
                             % (self.mini_batch_num, self.world))
        self.local_batch = self.mini_batch_num // self.world
        dev = self.device or torch.device("cuda", torch.cuda.current_device())
        self.engine = Engine(self.Ne, self.Nc, self.local_batch, variant=self.variant,
                             device=dev, batch_global=self.mini_batch_num, lr=self.lr,
                             process_group=self.pg)
        self._initialize()
        # fetchable attributes (filled by the last step, like sess.run results)
        self.C_edge_output2 = None
        self.C_edge_output2_logits = None
        self.loss_Hedge_mse = None
        self.loss_map = None
        self.loss_para = None
        # 0.001 * l2_loss(C_edge_output) (model_2.py:122): computed by the graph but fetched
        # by neither train nor test; here filled by test()'s forward launches
        self.loss_E_HR = None
        # the training sess.run fetches C_edge_output2 only (model_2.py:369-371); set True
        # to have train() also fill C_edge_output2_logits every step
        self.fetch_logits = False
        self.saver = Saver(self)

    def _initialize(self):
        """tf.global_variables_initializer(): truncated_normal(0.1) weights, zero biases,
        fresh Adam slots and beta powers."""
        self.engine.set_params(layout.init_flat(self.seed, self.variant))

    @property
    def vars(self):
        return layout.split(self.engine.get_params(), self.variant)

    @property
    def theta(self):
        return self.vars["map_conv/map_theta2:0"]

    # ------------------------------------------------------------------ data
    def _compact(self):
        """-> (C_edge_train, C_edge_test, train, test, maps).  'utils2': the reference's
        read_data 12-tuple through the bit-exact adapter; 'fast': hdgnn.loader reads the same
        files straight into the compact form (no dense arrays, no progress-bar sleeps)."""
        if self._given is not None:
            train, test, maps = self._given
            return onehot_relations(train.y), onehot_relations(test.y), train, test, maps
        if self.loader == "fast":
            from .loader import read_compact
            train, test, maps = read_compact(self.Repo, self.Step, self.Ne, self.Nc,
                                             self.mini_batch_num, root=self.data_root)
            return onehot_relations(train.y), onehot_relations(test.y), train, test, maps
        tup = self.reader(self, self.Step)
        train, test, maps = compact_from_read_data(tup, self.Ne, self.Nc, self.mini_batch_num)
        return np.asarray(tup[4]), np.asarray(tup[5]), train, test, maps

    def _device_batches(self, part, maps):
        """Per reference batch j: this rank's shard of commits j*mb .. (j+1)*mb with the
        maps of batch positions (model_2.py:365-381: Esc/Etc/..[:Mini_batch])."""
        out = []
        for (c0, c1), (p0, p1) in shard_plan(part.B, self.mini_batch_num, self.world, self.rank):
            sh = part.slice(c0, c1).with_maps(maps.slice(p0, p1))
            out.append(self.engine.upload(sh))
        return out

    def _gather(self, arr):
        """Concatenate a per-rank (lb, ...) array over ranks on every rank."""
        if self.world == 1:
            return arr
        import torch
        t = torch.from_numpy(np.ascontiguousarray(arr)).to(self.engine.device)
        parts = [torch.empty_like(t) for _ in range(self.world)]
        torch.distributed.all_gather(parts, t, group=self.pg)
        return torch.cat(parts).cpu().numpy()

    def _allsum(self, v):
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.engine.device)
        torch.distributed.all_reduce(t, group=self.pg)
        return t.item()

    # ------------------------------------------------------------------ train
    def _barrier(self):
        """Ranks meet before the first step and after rank 0's host work of an epoch, so no
        rank enters a data-parallel step far behind its peers (the xGMI exchange waits a
        bounded time for peer words)."""
        if self.world > 1:
            import torch
            torch.distributed.barrier(group=self.pg)

    def train(self, args):
        """model_2.py:335-424.  Every step's pre-update losses and top_ACC count land in its
        own row of an epoch buffer on the device (hdg_outputs.stats); at the epoch's end that
        buffer and the flat training state go to pinned host memory in two stream-ordered
        copies.  Epochs are pipelined one deep: epoch i+1 is enqueued before the host waits
        for epoch i, so epoch i's result line, result file and checkpoint (written by the
        saver thread through libhdgnn) overlap epoch i+1 on the GPU.  A split-mode exchange
        timeout (a step's update skipped, the fault count in every rank's stats) re-runs
        epoch i from the host copy of the state before it, with one block per commit
        (Engine.split_fault_retry); epochs of more than FAULT_POLL steps poll the fault
        slots every FAULT_POLL steps and stop a faulted epoch early."""
        import torch
        self._initialize()
        _, _, train, _, maps = self._compact()
        batches = self._device_batches(train, maps)
        nb = len(batches)
        counter = 1
        start_time1 = time.time()
        eng = self.engine
        S, dev = eng.state.numel(), eng.device
        th_off = layout.offsets(self.variant)["map_conv/map_theta2:0"][0]
        nr = max(nb, 1)
        # device stats rows and pinned host slots per epoch parity; host state slots mod 3
        # (a retry of epoch i needs the state after i-1 while i+1 is in flight)
        es = [torch.zeros(nr, _lib.STATS_LEN, dtype=torch.float32, device=dev) for _ in range(2)]
        hs = [torch.zeros(nr, _lib.STATS_LEN, dtype=torch.float32).pin_memory() for _ in range(2)]
        hst = [torch.zeros(S, dtype=torch.float32).pin_memory() for _ in range(3)]
        hst[2].copy_(eng.state)                          # "after epoch -1": the initial state
        outs = {}
        pflag = torch.zeros(2, dtype=torch.float32).pin_memory()   # fault-poll slots
        pdone = [torch.cuda.Event() for _ in range(2)]
        # per step row and epoch parity: the step with its ctypes arguments built once; the
        # epoch's host reads and completion events through libhdgnn (hipMemcpyAsync /
        # hipEvent: no dispatcher round per epoch)
        lib = eng.lib
        steps = [[eng.step_call(db, stats=es[p][j], logits=self.fetch_logits)
                  for j, db in enumerate(batches)] for p in range(2)]
        stream = eng._stream()
        done = [ctypes.c_void_p() for _ in range(2)]
        for ev in done:
            _lib.check(lib.hdg_event_create(ctypes.byref(ev)))
        rows_bytes, state_bytes = nr * _lib.STATS_LEN * 4, S * 4
        filepath = None
        if self.rank == 0:
            filepath = r'outputSelf/{}/model_{}/{}/result_{}.npy'.format(
                args.Repo, self.variant, self.Step, self.Step)
            os.makedirs(os.path.dirname(filepath), exist_ok=True)

        def launch(i):
            """Enqueue epoch i: its steps, then the host copies of its stats and end state.
            Split fused epochs of more than FAULT_POLL steps poll the fault slots every
            FAULT_POLL steps: the poll at step j copies the fault column so far to pinned
            memory, and waits only for the previous poll's copy (FAULT_POLL steps older), so
            the GPU keeps FAULT_POLL steps queued and the host is never in lockstep with it;
            a fault stops the epoch at the next poll after the one that saw it."""
            rows = es[i % 2]
            npoll = 0
            for j, step in enumerate(steps[i % 2]):
                step()
                if nb > FAULT_POLL and (j + 1) % FAULT_POLL == 0 and j + 1 < nb and \
                        eng.split and eng.path == _lib.PATH_FUSED:
                    if npoll:
                        pdone[(npoll - 1) % 2].synchronize()
                        if pflag[(npoll - 1) % 2].item() != 0.0:   # stop a faulted epoch early
                            rows[j + 1:].zero_()
                            rows[j + 1:, 7] = 1.0
                            break
                    pflag[npoll % 2:npoll % 2 + 1].copy_(rows[:j + 1, 7].amax().reshape(1),
                                                         non_blocking=True)
                    pdone[npoll % 2].record()
                    npoll += 1
            if nb and i == self.epoch - 1:              # the fetched outputs of the last step
                outs[i] = (eng.probs.clone(), eng.logits.clone() if self.fetch_logits else None)
            _lib.check(lib.hdg_memcpy_async(ctypes.c_void_p(hs[i % 2].data_ptr()),
                                            ctypes.c_void_p(rows.data_ptr()), rows_bytes, stream))
            _lib.check(lib.hdg_memcpy_async(ctypes.c_void_p(hst[i % 3].data_ptr()),
                                            ctypes.c_void_p(eng.state.data_ptr()), state_bytes,
                                            stream))
            _lib.check(lib.hdg_event_record(done[i % 2], stream))

        try:
            self._train_epochs(args, launch, done, hs, hst, outs, nb, th_off, counter, filepath)
        finally:
            for ev in done:
                lib.hdg_event_destroy(ev)
        end_time1 = time.time()
        if self.rank == 0:
            print('test time:' + str(end_time1 - start_time1))

    def _train_epochs(self, args, launch, done, hs, hst, outs, nb, th_off, counter, filepath):
        """train()'s epoch loop: epoch i+1 enqueued before the host waits for epoch i."""
        import torch
        eng, lib, dev = self.engine, self.engine.lib, self.engine.device
        self._barrier()
        if self.epoch > 0:
            launch(0)
        i = 0
        while i < self.epoch:
            if i + 1 < self.epoch and self.world == 1:
                launch(i + 1)
            _lib.check(lib.hdg_event_synchronize(done[i % 2]))
            host = hs[i % 2].numpy().astype(np.float64)
            if host[:nb, 7].any():                       # a split-mode exchange timed out
                torch.cuda.synchronize(dev)              # epoch i+1 (if launched) drained
                if eng.split and eng.path == _lib.PATH_FUSED and eng.split_fault_retry():
                    eng.restore(hst[(i - 1) % 3].numpy())
                    outs.pop(i + 1, None)
                    launch(i)
                    continue
                eng.check_status()
                raise RuntimeError("libhdgnn: a training step faulted (stats %s)" % host[:nb])
            if not np.isfinite(host[:nb, 0]).all():      # a NaN loss: a device fault (DP
                eng.check_status()                       # timeout) raises, a diverged run
                                                         # prints nan as the reference would
            tr_loss_Hedge = float(host[:nb, 0].sum())
            tr_loss_map = float(host[:nb, 1].sum())
            # the trailer's three 16-bit count parts per step, summed exactly in int64
            correct = int((np.rint(host[:nb, 4:7]).astype(np.int64) * _COUNT_W).sum())
            state = hst[i % 3].numpy()
            if nb:
                self.loss_Hedge_mse, self.loss_map, self.loss_para = (float(host[nb - 1, 0]),
                                                                      float(host[nb - 1, 1]),
                                                                      float(host[nb - 1, 2]))
                if i in outs:
                    self.C_edge_output2, self.C_edge_output2_logits = outs.pop(i)
            acc_top = correct / (nb * self.mini_batch_num * self.Ncr) if nb else 0.0
            # theta (model_2.py:369-371, 392): map_theta2 in the state after epoch i, as
            # self.theta reads it at this point
            theta = state[th_off:th_off + 2].astype(np.float32)
            resultString = "Epoch " + str(i + 1) + \
                           " acc: " + str(acc_top)[0:6] + \
                           " Hedge loss: " + str(tr_loss_Hedge / nb if nb else 0.0)[0:6] + \
                           " map MSE: " + str(tr_loss_map / nb if nb else 0.0)[0:6] + \
                           " theta: " + str(theta[0]) + ' ' + str(theta[1]) + '\n'
            if self.rank == 0:
                # appended by the writer thread, in order with the checkpoints (same bytes
                # as the reference's open(..., "a") + write per epoch)
                self.saver.writer().submit(text_path=filepath, text=resultString, append=True)
                print(resultString)
            counter += 1
            self.save(args.checkpoint_dir, counter, background=True, state=state)
            self._barrier()
            if self.world > 1 and i + 1 < self.epoch:   # DP: ranks launch in step after the barrier
                launch(i + 1)
            i += 1
        self.saver.flush()          # every epoch's files on disk before train() returns

    # sess.run's fetched C_edge_output2 / C_edge_output2_logits.  Training keeps the last
    # step's device output as a fresh tensor per epoch (later steps never change it) and
    # hands out a host numpy copy on first access, as sess.run returns one.
    def _fetched(self, key):
        f = self.__dict__.setdefault("_fetch", {})
        v = f.get(key)
        if v is not None and not isinstance(v, np.ndarray):
            v = f[key] = v.detach().cpu().numpy()
        return v

    @property
    def C_edge_output2(self):
        return self._fetched("probs")

    @C_edge_output2.setter
    def C_edge_output2(self, v):
        self.__dict__.setdefault("_fetch", {})["probs"] = v

    @property
    def C_edge_output2_logits(self):
        return self._fetched("logits")

    @C_edge_output2_logits.setter
    def C_edge_output2_logits(self, v):
        self.__dict__.setdefault("_fetch", {})["logits"] = v

    # ------------------------------------------------------------------ checkpoints
    def _model_dir(self, checkpoint_dir):
        return os.path.join(checkpoint_dir, "%s/model_%d/%s" % (self.Repo, self.variant, self.Step))

    def save(self, checkpoint_dir, step, background=False, state=None):
        """saver.save(sess, <dir>/g2g.model, global_step=step) (model_2.py:427-437): a TF V2
        bundle g2g.model-<step>.index / .data-00000-of-00001 under the TF variable names
        (hdgnn.tfckpt), plus TF1 Adam's slots and beta powers so training can resume, and
        the 'checkpoint' state file tf.train.get_checkpoint_state reads.  train() saves in
        the background (Saver.save(background=True)): the state is read at the epoch's end,
        the files are written while the next epoch runs, and train() flushes before it
        returns."""
        if self.rank != 0:
            return
        self.saver.save(self.sess, os.path.join(self._model_dir(checkpoint_dir), "g2g.model"),
                        global_step=step, background=background, state=state)

    def load(self, checkpoint_dir):
        """get_checkpoint_state + saver.restore (model_2.py:439-451).  Reads TF V2 bundles
        (this framework's or the reference's own; the latter carry no Adam slots, so the
        optimizer state is left as initialised) and this framework's older .npz files."""
        print(" [*] Reading checkpoint...")
        self.saver.flush()
        d = self._model_dir(checkpoint_dir)
        name = tfckpt.latest(d)
        if not name:
            return False
        path = os.path.join(d, name)
        if os.path.exists(path + ".index"):
            self.saver.restore(self.sess, path)
            return True
        if os.path.exists(path + ".npz"):
            z = np.load(path + ".npz", allow_pickle=False)
            flat = np.concatenate([np.asarray(z[n], np.float32).reshape(-1)
                                   for n, _ in layout.specs(self.variant)])
            m, v, bp = ((z["_adam_m"], z["_adam_v"], z["_beta_pow"]) if "_adam_m" in z
                        else (None, None, None))
        else:
            return False
        import torch
        eng = self.engine
        eng.set_params(flat)
        if m is not None:
            eng.m.copy_(torch.from_numpy(np.asarray(m, np.float32)))
            eng.v.copy_(torch.from_numpy(np.asarray(v, np.float32)))
            eng.beta_pow.copy_(torch.from_numpy(np.asarray(bp, np.float32)))
        return True

    # ------------------------------------------------------------------ test
    def test(self, args):
        _, C_edge_test, _, test, maps = self._compact()
        self._initialize()
        checkpoint_dir = os.path.join(self.checkpoint_dir, self.Repo)
        if self.load(checkpoint_dir):
            print(" [*] Load SUCCESS")
        else:
            print(" [!] Load failed...")
        te_loss_Hedge = 0.0
        te_loss_map = 0.0
        C_edge_t = []
        eng = self.engine
        start_time = time.time()
        end_time = start_time
        for db in self._device_batches(test, maps):
            probs, logits, ce_sum = eng.forward(db)
            p = probs.cpu().numpy()
            self.C_edge_output2_logits = logits.clone()     # not overwritten by later batches
            self.loss_E_HR = self._allsum(float(eng.ehr.item()))
            eng.check_status()
            ce = self._allsum(float(ce_sum.item())) / (self.mini_batch_num * self.Ncr)
            th1 = self.vars["map_conv/map_theta1:0"].reshape(-1).astype(np.float64)
            th2 = self.vars["map_conv/map_theta2:0"].reshape(-1).astype(np.float64)
            lmap = 0.01 * (np.sqrt((th2 ** 2).sum()) + np.sqrt((th1 ** 2).sum()))
            end_time = time.time()
            te_loss_Hedge += ce
            te_loss_map += lmap
            self.C_edge_output2 = p
            C_edge_t.append(self._gather(p))
        n_used = len(C_edge_t) * self.mini_batch_num
        C_edge_t1 = (np.array(C_edge_t).reshape(n_used, self.Dr, self.Ncr) if C_edge_t
                     else np.zeros((0, self.Dr, self.Ncr), np.float32))
        if self.rank != 0:
            return
        step_dir = 'outputSelf/%s/model_%d/%s/' % (args.Repo, self.variant, self.Step)
        os.makedirs(step_dir, exist_ok=True)
        np.save(step_dir + 'C_edge_t' + str(self.Ne) + '.npy', C_edge_t1)
        np.save(step_dir + 'C_edge_y' + str(self.Ne) + '.npy',
                C_edge_test.reshape(len(C_edge_test), self.Dr, self.Ncr))
        ev = _evaluation_funcs()
        C_edge_t2 = ev.process_edge(C_edge_t1)
        C_edge_y = C_edge_test[:n_used]
        print('topol_acc: ' + str(ev.top_ACC(C_edge_y, C_edge_t2)))
        print('prec: ' + str(ev.prec(C_edge_y, C_edge_t2)))
        print('recall: ' + str(ev.recall(C_edge_y, C_edge_t2)))
        print('F1-score: ' + str(ev.f1(C_edge_y, C_edge_t2)))
        print('AUC-score: ' + str(ev.AUC(C_edge_y, C_edge_t2)))
        print('test time:' + str(end_time - start_time))
