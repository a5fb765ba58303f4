import torch, os
print("backend", torch.cuda.get_allocator_backend())
print("conf", os.environ.get("PYTORCH_HIP_ALLOC_CONF"), os.environ.get("PYTORCH_CUDA_ALLOC_CONF"))
x = torch.empty((4096, 12, 131072), dtype=torch.uint8, device="cuda")
print("ptr", hex(x.data_ptr()), x.data_ptr() % (1 << 21), x.data_ptr() % (1 << 30))
print(torch.cuda.memory_stats().get("num_alloc_retries"), torch.cuda.memory_reserved())
