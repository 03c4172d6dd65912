import torch, time
x = torch.empty(205_520_896, dtype=torch.bfloat16, device="cuda")  # 411 MB = the stem output at bs=256
for _ in range(3): x.fill_(1.0)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20): x.fill_(1.0)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(f"fill 411 MB: {ms*1e3:.1f} us = {411e6/ms/1e9:.2f} TB/s")
y = torch.empty_like(x)
e0.record()
for _ in range(20): y.copy_(x)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(f"copy 411 MB: {ms*1e3:.1f} us = {822e6/ms/1e9:.2f} TB/s (read+write)")
