"""The roofline numerator and the product-count pricing of kernel variants
(hkv/opcount.py)."""
from hkv import opcount as oc


def test_frozen_reference_numerator():
    assert oc.P_ALG_ECMULT == 103553


def test_implementation_count_is_the_default_build():
    # radix-16 Q windows, beta * x stored per table entry (hkv_layout.h HKV_QW = 4)
    assert oc.QW == 4
    assert oc.ecmult_products() == oc.ECMULT_PRODUCTS_PER_VERIFY == 123582


def test_radix32_xy_table_saves_under_two_percent():
    """radix-32 windows with an (x, y)-only 16-entry
    table forming beta * x per lambda addition. The doubled per-signature
    table build eats the 14 saved additions; against radix 16 with its top
    two windows merged (HKV_TOP_MERGE) the (x, y)-only table costs more
    products and the stored-beta one saves 0.5 %, below the 2% adoption bar
    before any memory effect, so neither is built."""
    base = oc.ecmult_products()
    xy32 = oc.ecmult_products(5, beta_per_lookup=True)
    stored32 = oc.ecmult_products(5, beta_per_lookup=False)
    assert xy32 > base and stored32 < base
    assert (base - stored32) / base < 0.02
