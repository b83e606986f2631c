import torch, time
ys = torch.empty((1 << 20) * 16384, dtype=torch.uint8, device="cuda")
for _ in range(2): ys.fill_(1)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); 
for _ in range(3): ys.fill_(2)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 3
print("fill 16 GiB: %.2f ms, %.2f TB/s" % (ms, ys.numel() / ms / 1e9))
v = ys.view(torch.int64)
e0.record()
for _ in range(3): v.copy_(v.flip(0)) if False else v.mul_(1)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 3
print("rmw 16 GiB: %.2f ms, %.2f TB/s (r+w)" % (ms, 2 * ys.numel() / ms / 1e9))
