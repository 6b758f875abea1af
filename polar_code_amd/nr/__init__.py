"""NR front-ends.  Only the polar chain is on the hot path; the reference's NR LDPC demo
(dl_scl_polar/nr/ldpc) is out of scope."""
