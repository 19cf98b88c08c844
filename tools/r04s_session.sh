# flag-variant parity subset + A/B against the saved base library, then the full validation (r04q) on the in-tree library
bash tools/r04r_session.sh && bash tools/r04q_session.sh
