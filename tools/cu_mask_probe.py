"""Map CU-mask bits to XCDs: launch a probe grid on streams masked by each
DML_CU_MASK pattern part (parallel/cu_mask.py) and count the distinct XCDs /
CUs its blocks ran on.  python tools/cu_mask_probe.py [--out file.json]"""
import argparse, ctypes as C, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_machine_learning_amd.parallel import cu_mask

ap = argparse.ArgumentParser(); ap.add_argument("--out", default=""); args = ap.parse_args()
P = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libxcd_probe.so"))
P.xcd_probe.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
dev = torch.device("cuda", 0)
ncu = cu_mask.num_cus()
B = 4096
res = {"ncu": ncu}
cases = [("none", None)] + [(f"{p}:{k}", cu_mask.mask_words(p, k, ncu)) for p in ("lohi", "mod8", "evenodd") for k in (0, 1)]
cases += [(f"bit{i}", [(1 << (i % 32)) if w == i // 32 else 0 for w in range((ncu + 31) // 32)]) for i in (0, 1, 2, 7, 8, 31, 32, 64, 128)]
for name, words in cases:
    ms = cu_mask.MaskedStream(dev, words) if words else None
    s = ms.stream if ms else torch.cuda.current_stream(dev)
    out = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    assert P.xcd_probe(out.data_ptr(), B, s.cuda_stream) == 0
    s.synchronize()
    v = out.view(B, 2).cpu().tolist()
    xccs = sorted({a for a, _ in v})
    cus = sorted({(a, (h >> 8) & 0xF, (h >> 12) & 0x3, (h >> 13) & 0x7) for a, h in v})  # xcc, cu, sh, se (raw fields)
    res[name] = {"xccs": xccs, "n_cu_ids": len(cus), "blocks_per_xcc": {x: sum(1 for a, _ in v if a == x) for x in xccs}}
    print(name, res[name], flush=True)
if args.out:
    json.dump(res, open(args.out, "w"), indent=1)
