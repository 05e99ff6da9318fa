"""Per-tensor gradient error of one fp32 trainer step against the oracle (debug aid)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

from test_gpu_train import _batch, _models, _oracle_step, LR, BETAS  # noqa: E402
from _cases import rel  # noqa: E402


def main():
    for rep in range(3):
        one(rep)


def one(rep):
    import tpgan_train
    from oracle import tpgan_oracle as O
    gpu = torch.device("cuda", 0)
    G, D = _models(gpu)
    tr = tpgan_train.TPGANTrainer(G, D, lr=LR, betas=BETAS, compute_dtype=torch.float32, use_dropout=False)
    b = _batch(2)
    bg = {k: (v.float() if v.is_floating_point() else v).to(gpu) for k, v in b.items()}
    tr._phase_a(bg)
    torch.cuda.synchronize()
    PG, PD = O.make_params(torch.float64)
    for p in PD.values():
        p.requires_grad_(True)
    fake = O.generator(PG, b["I128"], b["left_eye"], b["right_eye"], b["nose"], b["mouth"], b["z"])[0]
    d = O.discriminator(PD, torch.cat([b["frontal"], fake], 0))
    loss = d[2:].mean() - d[:2].mean()
    gD = torch.autograd.grad(loss, list(PD.values()))
    print("fake rel", rel(tr._st["outs"][0].detach().cpu(), fake.detach()))
    def show(tag):
        torch.cuda.synchronize()
        errs = [(k, rel(p.grad.detach().cpu(), gr), float(gr.norm())) for (k, p), gr in zip(D.named_parameters(), gD)]
        allm = torch.cat([p.grad.detach().double().cpu().reshape(-1) for p in D.parameters()])
        allr = torch.cat([g.reshape(-1) for g in gD])
        print(tag, "global %.3e" % rel(allm, allr), "worst", max(errs, key=lambda e: e[1]))
    show("rep %d after A" % rep)



if __name__ == "__main__":
    main()
