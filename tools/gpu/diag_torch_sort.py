import torch
d = torch.device("cuda")
for n in [30_000_000, 34_000_000, 100_000_000]:
    g = torch.Generator(device=d); g.manual_seed(1)
    x = torch.randint(-2**62, 2**62, (n,), device=d, generator=g)
    for stable in (True, False):
        idx = torch.argsort(x, stable=stable)
        perm = bool((torch.bincount(idx, minlength=n) == 1).all())
        srt = bool((x[idx][1:] >= x[idx][:-1]).all())
        print(n, "stable" if stable else "unstable", "perm", perm, "sorted", srt, flush=True)
    s = torch.arange(n // 16384 + 1, device=d)
    r = torch.repeat_interleave(s, torch.full((s.numel(),), 16384, device=d))
    print(n, "repeat_interleave ok", bool((r == torch.arange(r.numel(), device=d) // 16384).all()), flush=True)
