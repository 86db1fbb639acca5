"""Which kernel a forced autotuner candidate must launch (artsbir_last_kernel()).

A candidate forced through ARTSBIR_PGEMM_CFG / ARTSBIR_WGRAD_CFG that does not
take a shape leaves the launch to the library's fallback; a forced-candidate
test must then be reported as skipped, never pass on a kernel other than the one
it names (round-4 review: candidate "23" silently re-tested the fallback)."""
import re

import pytest

import _hip

CONV = {
    "-2": r"conv_gemm_kernel<",
    "0": r"pgemm_kernel<256,256(,bnb)?>$",
    "1": r"pgemm_kernel<256,128(,bnb)?>$",
    "2": r"pgemm_kernel<256,64(,bnb)?>$",
    "3": r"pgemm_kernel<128,128(,bnb)?>$",
    "4": r"pgemm_kernel<256,32(,bnb)?>$",
    "5": r"pgemm_kernel<256,256,k32(,bnb)?>$",
    "10": r"pstream_kernel<(32|64|128)(,bnb)?>$",
    "11": r"pgemm_kernel<256,128(,bnb)?,pf>$",
    "12": r"pgemm_kernel<256,64(,bnb)?,pf>$",
    "13": r"pgemm_kernel<128,128(,bnb)?,pf>$",
    "14": r"pstream_kernel<(64|128),bnbk>$",
    "15": r"pstream_kernel<(64|128),k32>$",
    "16": r"pgemm_kernel<128,128,k32,glb(,bnb)?>$",
    "18": r"pgemm_kernel<256,128,k32,glb,bnb>$",
    "19": r"pgemm_kernel<256,128,k32,glb>$",
    "20": r"sconv_kernel<",
    "21": r"hconv_kernel<",
    "22": r"pp256_kernel(<bnb>)?$",
    "24": r"pstream_kernel<(32|64|128),nt>$",
    "25": r"pstream_kernel<(64|128),k32,nt>$",
    "26": r"rstream_kernel<bnb(,two)?>$",
}


def wgrad_pattern(cfg: str) -> str:
    c = int(cfg)
    if c == -1:
        return r"wgrad_kernel<"
    if c >= 100:
        return r"pw256_kernel<"
    if c >= 36:
        return r"hwgrad_kernel<"
    return r"pwgrad_kernel<"


def last_kernel() -> str:
    return _hip.lib().artsbir_last_kernel().decode()


def require(cfg: str, wgrad: bool = False) -> str:
    """skip unless the forced candidate cfg is the kernel that just ran"""
    name = last_kernel()
    if cfg == "auto":
        return name
    pat = wgrad_pattern(cfg) if wgrad else CONV[cfg]
    if not re.match(pat, name):
        pytest.skip(f"candidate {cfg} does not take this case (the fallback ran {name})")
    return name
