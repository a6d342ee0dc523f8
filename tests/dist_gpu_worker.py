"""Worker of tests/test_gpu_distributed.py: one rank of a world-2 job on ONE GPU over gloo (RCCL
refuses two ranks per device), launched by torch.distributed.run. It runs the product's
multi-GPU path -- build_index_sharded over the B/32 encoder (encode_items / rebuild_index) and
ShardedIndex over CosineIndex with the GPU top-k merge -- and rank 0 compares every result with
the single-rank computation, writing a JSON verdict."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import clip_lora_match_amd as clm  # noqa: E402
from clip_lora_match_amd import synthetic as syn  # noqa: E402
from clip_lora_match_amd import weights as W  # noqa: E402
from clip_lora_match_amd.distributed import ShardedIndex, merge_topk_gpu  # noqa: E402
from clip_lora_match_amd.engine import ClipLoraModel  # noqa: E402
from clip_lora_match_amd.index_build import _f16_exchange, _f16_restore, _renormalize, encode_items, rebuild_index  # noqa: E402
from clip_lora_match_amd.processor import ClipProcessor  # noqa: E402
from clip_lora_match_amd.search import CosineIndex  # noqa: E402


def main(out_path, tmpdir):
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    res = {"world": world}
    cfg = clm.get_preset("ViT-B/32")
    model = ClipLoraModel(cfg, compute_dtype="float16", max_batch=8)
    model.load_tensors(W.synthetic_state_dict(cfg, 0))
    model.load_tensors(W.synthetic_lora(cfg, 1))
    model.finalize()
    proc = ClipProcessor(cfg)
    # 1. sharded index build (images and captions), 37 items in batches of 8
    imgs = list(syn.images_u8(37, cfg.image_size, 300))
    caps = [list(map(int, r)) for r in syn.captions(37, cfg.max_pos, cfg.bos_token_id, cfg.eos_token_id, 301)]
    e_img = encode_items(model, proc, images=imgs, batch_size=8)
    e_txt = rebuild_index(model, proc, caps, [f"img{i}.jpg" for i in range(37)], os.path.join(tmpdir, "idx.pt"),
                          batch_size=8)
    # every rank may read the file right after rebuild_index returns
    obj = torch.load(os.path.join(tmpdir, "idx.pt"), map_location="cpu", weights_only=True)
    fr = torch.tensor([int(obj["embeddings"].shape[0])])
    lo, hi = fr.clone(), fr.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    res["file_rows_min_max"] = [int(lo), int(hi)]
    # 2. row-sharded search: 300k fp32 rows, each rank holds its shard_range
    n, dim, nq, k = 300_000, 512, 24, 10
    rows = syn.gaussian_rows(n, dim, 41, fp16=False)
    qs = syn.gaussian_rows(nq, dim, 42, fp16=False)
    qs[:4] = rows[[5, 150_000, 150_001, 299_999]]
    sh = ShardedIndex(dim, n)
    sh.append_shard(torch.from_numpy(rows[sh.start:sh.stop]))
    s_sh, i_sh = sh.search(torch.from_numpy(qs), k)
    # 3. configs[2] in miniature: 64k device-generated images (seeded by global row), sharded build
    #    through rebuild_index(from_images=True) with the .pt write; rank 0 redoes it unsharded with
    #    another batch size (row results must not depend on the batch split)
    n_big = 65_536
    big = ClipLoraModel(cfg, compute_dtype="bfloat16", max_batch=256)
    big.load_tensors(W.synthetic_state_dict(cfg, 0))
    big.load_tensors(W.synthetic_lora(cfg, 1))
    big.finalize()
    src = syn.DeviceImages(n_big, cfg.image_size, seed=2024)
    names = [f"synthetic/{i:06d}.png" for i in range(n_big)]
    e_big = rebuild_index(big, proc, [""] * n_big, names, os.path.join(tmpdir, "big.pt"), batch_size=256,
                          from_images=True, images=src)
    # the fp16 all_gather exchange (half the link bytes): the fp32 rows rounded to fp16 and
    # re-normalised in fp32 after the gather, on every rank
    e_big16 = rebuild_index(big, proc, [""] * n_big, names, os.path.join(tmpdir, "big16.pt"), batch_size=256,
                            from_images=True, images=src, exchange="fp16", host_rows=False)
    big_file = torch.load(os.path.join(tmpdir, "big.pt"), map_location="cpu", weights_only=True)
    # 4. a failed write on rank 0 raises on every rank (nobody is left in a collective)
    blocker = os.path.join(tmpdir, "not_a_dir")
    if rank == 0:
        open(blocker, "w").close()
    dist.barrier()
    try:
        rebuild_index(model, proc, caps[:4], ["a", "b", "c", "d"], os.path.join(blocker, "idx.pt"), batch_size=8)
        raised = False
    except RuntimeError as e:
        raised = "rank 0 failed to write" in str(e) or rank == 0
    except OSError:
        raised = rank == 0   # rank 0 itself sees the OSError from mkdir
    flag = torch.tensor([int(raised)])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    res["write_failure_raised_everywhere"] = bool(flag.item())
    dist.barrier()
    if rank == 0:
        ref_big = torch.cat([_renormalize(big.encode_pixels(src.batch(a, min(a + 200, n_big))))
                             for a in range(0, n_big, 200)]).cpu()
        res["big_build_equal"] = bool(torch.equal(e_big, ref_big))
        res["big_f16_exchange_equal"] = bool(torch.equal(e_big16.cpu(), _f16_restore(_f16_exchange(ref_big.cuda())).cpu()))
        res["big_f16_exchange_device"] = str(e_big16.device)
        res["big_file_equal"] = bool(torch.equal(big_file["embeddings"], ref_big))
        res["big_file_rows"] = int(big_file["embeddings"].shape[0])
        res["big_paths_ok"] = big_file["image_paths"][12345] == names[12345]
        # the synthetic source is deterministic per global row, whatever the split
        res["synth_rows_stable"] = bool(torch.equal(src.batch(1000, 1003).cpu(),
                                                    torch.cat([src.batch(1000, 1001), src.batch(1001, 1003)]).cpu()))
        # single-rank references
        # (encode_items re-normalises each row once more, as rebuild_index.py:72 does)
        ref_img = torch.cat([_renormalize(model.encode_pixels(torch.from_numpy(np.stack(imgs[a:a + 8])).cuda()))
                             for a in range(0, 37, 8)]).cpu()
        ref_txt = torch.cat([_renormalize(model.encode_ids(proc.token_ids(caps[a:a + 8]).cuda()))
                             for a in range(0, 37, 8)]).cpu()
        res["build_img_equal"] = bool(torch.equal(e_img.cpu(), ref_img))
        dimg = (e_img.cpu().float() - ref_img.float()).abs()
        res["build_img_maxdiff"] = float(dimg.max())
        res["build_img_rows_differing"] = torch.nonzero(dimg.amax(1) > 0).flatten().tolist()
        res["build_txt_equal"] = bool(torch.equal(e_txt, ref_txt))
        res["file_equal"] = bool(torch.equal(obj["embeddings"], ref_txt))
        one = CosineIndex(dim, capacity=n)
        one.append(torch.from_numpy(rows))
        s1, i1 = one.search(torch.from_numpy(qs), k)
        res["search_idx_equal"] = bool(torch.equal(i_sh, i1))
        res["search_scores_equal"] = bool(torch.equal(s_sh, s1))
        res["planted_top1"] = i_sh[:4, 0].tolist()
        # merge kernel alone: two halves of one list merge back to the list
        s2, i2 = merge_topk_gpu(torch.cat([s1[:, :5], s1[:, 5:]], 1), torch.cat([i1[:, :5], i1[:, 5:]], 1), 2, k)
        res["merge_roundtrip"] = bool(torch.equal(i2, i1) and torch.equal(s2, s1))
        json.dump(res, open(out_path, "w"))
    dist.barrier()
    big.close()
    model.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
