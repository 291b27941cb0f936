# diagnostic variant: up to 16 launch slices per work unit (the product caps at 8)
s|std::min<long long>(8, 0x7FFFFFFFll / std::max(nq, 1ll))|std::min<long long>(16, 0x7FFFFFFFll / std::max(nq, 1ll))|
