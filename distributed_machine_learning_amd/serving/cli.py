"""The interactive command surface (reference worker.py:1629-2034, menu 1641-1672).

Kept command-for-command:
  C1                      query count + query rate over the last 10 s, per model
  C2                      per-image processing time: mean, stdev, quartiles (+ p50/p90/p99)
  C3 <model> <batch>      set the per-model batch size on the coordinator
  submit-job <model> <N>  (C4) submit a job; prints the job id
  get-output <jobid>      (C4) final_<jobid>.json: the rank service's coordinator renders it from the
                          top-5 rows gathered over the data group; else merge output_<jobid>_*.json
  C5 [n [job]]            current assignments {worker: {model, job_id, batch_id}}; on the rank
                          service also the last n completed batches with the rank that ran each
  predict-locally <model> <jobid> <N|[a.jpeg,b.jpeg]>
  put <local> <sdfs> | get <sdfs> <local> | get-all <pattern> <dir> | delete <sdfs>
  ls <sdfs> | ls-all <pattern> | store | get-versions <sdfs> <n> <local>
  1..8  membership, self id, join, leave, load testfiles, per-node files, all files, file count
  9, 10 (test mode) bytes/s sent, false-positive rate
Every command returns its text (the reference printed); ``run_line`` is what
the stdin loop and ``--cmd`` scripts call.
"""
from __future__ import annotations

import ast
import glob
import json
import os
import random
import time
from typing import List

from ..cluster.frames import MsgType
from .node import Node

MENU = """MP4-compatible commands:
 C1: Query Rate (10sec) & Query Count [Per model]
 C2: Query Processing Time: [Average, Percentiles, Standard Deviation]
 C3 <InceptionV3|ResNet50> <Batch Size>
 C4: submit-job <InceptionV3|ResNet50> <num:of images>
 C4: get-output <jobid>
 C5: Display current assigned jobs
 predict-locally <model> <jobid> <N|[list]>
options:
 1. list the membership list.   2. list self id.   3. join the group.   4. leave the group.
 5. load testfiles into sdfs.   6. print files stored per node.   7. print all files in the SDFS.
 8. print number of files in the SDFS.   9. print current bps (test mode).   10. false positive rate (test mode).
commands:
 put <local> <sdfs> | get <sdfs> <local> | get-all <pattern> <local_dir> | delete <sdfs>
 ls <sdfs> | ls-all <pattern> | store | get-versions <sdfs> <numversions> <local>"""


class Cli:
    def __init__(self, node: Node, testfiles: str = "", download_dir: str = "./download"):
        self.node = node
        self.testfiles = testfiles or os.environ.get("DML_TESTFILES", "")
        self.download_dir = download_dir

    async def run_line(self, line: str) -> str:
        parts = line.strip().split()
        if not parts:
            return ""
        cmd, args = parts[0], parts[1:]
        t0 = time.monotonic()
        try:
            out = await self._dispatch(cmd, args)
        except (IndexError, ValueError) as e:
            out = f"bad arguments for {cmd}: {e}\n{MENU}"
        return f"{out}\n[{cmd} took {time.monotonic() - t0:.3f}s]"

    async def _dispatch(self, cmd: str, a: List[str]) -> str:
        n = self.node
        c = cmd.upper()
        if c in ("HELP", "MENU", "?"):
            return MENU
        if c == "C1":
            r = await n.leader_request(MsgType.GET_C1_COMMAND)
            return "leader unreachable" if r is None else json.dumps(r.payload["c1"], indent=2)
        if c == "C2":
            r = await n.leader_request(MsgType.GET_C2_COMMAND)
            return "leader unreachable" if r is None else json.dumps(r.payload.get("detail", r.payload), indent=2)
        if c == "C3":
            r = await n.leader_request(MsgType.SET_BATCH_SIZE, {"model": a[0], "batch_size": int(a[1])})
            return "leader unreachable" if r is None else f"batch size of {a[0]} set to {a[1]}"
        if c == "C5":
            # "C5" / "C5 <n>" / "C5 <n> <job>": the running assignments, plus (rank service) the
            # last n completed batches with the rank that ran each and its output file
            req = {"history": int(a[0]) if a else 16}
            if len(a) > 1:
                req["job_id"] = int(a[1])
            r = await n.leader_request(MsgType.GET_ASSIGNMENTS, req)
            if r is None:
                return "leader unreachable"
            out = json.dumps(r.payload["assignments"], indent=2)
            if r.payload.get("history"):
                out += "\nrecent batches:\n" + "\n".join(
                    f"  job {e['job_id']} batch {e['batch_id']} ({e['model']}) ran on rank {e['rank']} -> {e['output']}"
                    for e in r.payload["history"])
            return out
        if cmd == "submit-job":
            jid = await n.submit_job(a[0], int(a[1]))
            return "submit failed (no leader)" if jid is None else f"submitted job {jid}"
        if cmd == "wait-job":
            ok = await n.wait_job(int(a[0]), float(a[1]) if len(a) > 1 else 600.0)
            return f"job {a[0]} {'finished' if ok else 'not finished'}"
        if cmd == "get-output":
            p = await n.get_output(int(a[0]), self.download_dir)
            return f"no outputs for job {a[0]}" if p is None else f"merged into {p}"
        if cmd == "predict-locally":
            return await self._predict_locally(a)
        if cmd == "put":
            ok, err = await n.store.put_file(a[0], a[1])
            return f"put {a[1]}: {'ok' if ok else 'FAILED ' + err}"
        if cmd == "get":
            got = await n.store.get(a[0])
            if got is None:
                return f"{a[0]} not found"
            with open(a[1], "wb") as f:
                f.write(got[1])
            return f"got {a[0]} v{got[0]} -> {a[1]}"
        if cmd == "get-all":
            names = await n.store.ls_all(a[0])
            os.makedirs(a[1], exist_ok=True)
            for name in names:
                got = await n.store.get(name)
                if got:
                    with open(os.path.join(a[1], name), "wb") as f:
                        f.write(got[1])
            return f"downloaded {len(names)} files into {a[1]}"
        if cmd == "delete":
            ok, err = await n.store.delete(a[0])
            return f"delete {a[0]}: {'ok' if ok else 'FAILED ' + err}"
        if cmd == "ls":
            return f"{a[0]}: {await n.store.ls(a[0])}"
        if cmd == "ls-all":
            return "\n".join(await n.store.ls_all(a[0] if a else "*"))
        if cmd == "store":
            return json.dumps(n.local.all_files(), indent=2)
        if cmd == "get-versions":
            vers = await n.store.get_versions(a[0], int(a[1]))
            with open(a[2], "wb") as f:
                for v, data in vers:
                    f.write(f"----- {a[0]} version {v} -----\n".encode())
                    f.write(data)
                    f.write(b"\n")
            return f"wrote {len(vers)} versions of {a[0]} to {a[2]}"
        if cmd == "1":
            return json.dumps(n.ml.table(), indent=2)
        if cmd == "2":
            return f"{n.name} (incarnation {n.ml.me.incarnation}, role {n.cfg.role}, leader {n.leader()})"
        if cmd == "3":
            n.fd.enabled = True
            await n.join()
            return "joined"
        if cmd == "4":
            await n.fd.leave()
            return "left the group"
        if cmd == "5":
            return await self._load_testfiles(a[0] if a else self.testfiles)
        if cmd == "6":
            return json.dumps(n.local.all_files(), indent=2)
        if cmd == "7":
            if n.is_leader():
                return json.dumps(n.store.meta.file_map, indent=2)
            return "\n".join(await n.store.ls_all("*"))
        if cmd == "8":
            return str(len(await n.store.ls_all("*")))
        if cmd == "9":
            t = n.transport
            bps = t.bps() if hasattr(t, "bps") else t.bytes_sent / max(1e-9, time.monotonic() - n.started_at)
            return f"{bps:.1f} bytes/s sent"
        if cmd == "10":
            return f"false positive rate {n.ml.false_positive_rate():.4f} ({n.ml.false_positives}/{n.ml.suspicions})"
        return f"unknown command {cmd}\n{MENU}"

    async def _load_testfiles(self, path: str) -> str:
        files = sorted(glob.glob(os.path.join(path, "*.jpeg")) + glob.glob(os.path.join(path, "*.jpg")))
        ok = 0
        for f in files:
            good, _ = await self.node.store.put_file(f, os.path.basename(f))
            ok += good
        return f"loaded {ok}/{len(files)} files from {path} into the store"

    async def _predict_locally(self, a: List[str]) -> str:
        """Run the local backend on N random files (or a list) from the test folder
        (reference worker.py:1891-1925)."""
        model, jid, spec = a[0], int(a[1]), " ".join(a[2:])
        files = sorted(glob.glob(os.path.join(self.testfiles, "*.jpeg")))
        if spec.startswith("["):
            names = ast.literal_eval(spec) if "'" in spec or '"' in spec else spec.strip("[]").split(",")
            paths = [os.path.join(self.testfiles, s.strip()) for s in names]
        else:
            paths = random.sample(files, min(int(spec), len(files)))
        be = self.node.worker.backend if self.node.worker else None
        if be is None:
            from .inference import CpuBackend

            be = CpuBackend()
        blobs = [open(p, "rb").read() for p in paths]
        arr = be.decode_batch(model, blobs)
        idx, prob = be.predict(model, arr)
        from .output import decode_top5, output_name, write_output

        os.makedirs(self.download_dir, exist_ok=True)
        out = os.path.join(self.download_dir, output_name(jid, 0, self.node.name.replace(":", "_")))
        write_output(out, decode_top5(paths, idx, prob))
        return f"predicted {len(paths)} images -> {out}"
