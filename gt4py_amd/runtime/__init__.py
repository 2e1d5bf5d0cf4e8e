"""Native runtime of gt:mi355x: hipcc JIT cache, C-ABI loader, device/stream helpers."""
