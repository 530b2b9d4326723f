import os, sys, socket, torch, torch.distributed as dist, torch.multiprocessing as mp
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import test_tp_gpu as T

def worker(rank, world, port, q, rows, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DLMS_XGMI_SLAB_MB="8")
    if mode == "nograph_prefill":
        os.environ["DLMS_PREFILL_GRAPH"] = "0"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    cfg, w, prompts = T._setup("124m-2l", rows)
    eng = HipGPT2Engine(cfg, w, max_batch=rows, max_length=64, tp_group=dist.group.WORLD, use_graph=mode != "eager", p2p=True)
    outs = [eng.generate(prompts) for _ in range(3)]
    q.put((rank, outs))
    dist.destroy_process_group()

if __name__ == "__main__":
    rows = int(sys.argv[1]); mode = sys.argv[2]
    ctx = mp.get_context("spawn"); q = ctx.Queue()
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ps = [ctx.Process(target=worker, args=(r, 8, port, q, rows, mode)) for r in range(8)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=300) for _ in range(8))
    [p.join(60) for p in ps]
    outs = res[0]
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    cfg, w, prompts = T._setup("124m-2l", rows)
    ref = HipGPT2Engine(cfg, w, max_batch=rows, max_length=64, use_graph=False).generate(prompts)
    print(mode, rows, "runs equal:", [outs[i] == outs[0] for i in range(3)], "1==2:", outs[1] == outs[2],
          "ranks equal:", all(res[r] == outs for r in range(8)), "run==tp1:", [o == ref for o in outs], flush=True)
    for i in range(3):
        d = [(b, len(prompts[b]), next((j for j, (x, y) in enumerate(zip(ref[b], outs[i][b])) if x != y), None))
             for b in range(rows) if ref[b] != outs[i][b]]
        print(" RUN", i, "vs tp1 (row, prompt len, first diff pos):", d[:10], flush=True)
