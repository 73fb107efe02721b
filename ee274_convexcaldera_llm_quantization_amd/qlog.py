"""The reference quantiser's one host side effect, shared by the drop-in LowMemoryQuantizer
and the engine: every bbint4/bbint2 call appends one CSV row [id(quantizer), number of
outliers] to ./outlier_log.csv (RCR/src/caldera/utils/quantization.py:122-133, :190-199)."""
import csv
import os


def log_outliers(qid: int, n: int, log_file: str = "outlier_log.csv"):
    if not os.path.exists(log_file):
        with open(log_file, mode="w", newline="") as f:
            csv.writer(f).writerow(["Call_ID", "Num_Outliers"])
    with open(log_file, mode="a", newline="") as f:
        csv.writer(f).writerow([qid, n])


def check_method_bits(method: str, bits: int):
    """The constructor checks of LowMemoryQuantizer (quantization.py:20-43, :38-54)."""
    assert bits in (2, 4, 8, 16), "Bit-width not supported!"
    if method not in ("uniform", "nf4", "nf2", "bbint4", "bbint2"):
        raise NotImplementedError(f"Quantization method '{method}' not supported yet.")
    if method == "nf4" and bits != 4:
        raise ValueError("NF4 quantization supports only 4 bits.")
    if method == "nf2" and bits != 2:
        raise ValueError("NF2 quantization supports only 2 bits.")
    if method == "bbint4" and bits != 4:
        raise ValueError("bbint4 quantization supports only 4 bits.")


def code_bits(method: str, bits: int) -> int:
    """Bits per stored code: nf4/bbint4 4, nf2/bbint2 2 (bbint2 packs 2-bit codes whatever
    num_bits says, quantization.py:218-221), uniform its num_bits."""
    return {"nf4": 4, "nf2": 2, "bbint4": 4, "bbint2": 2}.get(method, bits)
