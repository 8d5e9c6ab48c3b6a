import time, torch
ss = [torch.cuda.Stream() for _ in range(4)]
for s in ss:
    with torch.cuda.stream(s):
        (torch.ones(1 << 20, device="cuda") * 2).sum().item()
torch.cuda.synchronize()
print("holding", flush=True)
time.sleep(75)
