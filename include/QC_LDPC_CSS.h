// QC_LDPC_CSS.h -- the quasi-cyclic CSS code generator of QEC_LDPC/QC_LDPC_CSS.h /
// QEC_LDPC/QEC_LDPC_CSS.cu:5-131 (construction of arXiv:quant-ph/0701020), as a
// factory for Quantum_LDPC_Code.  The reference's version is commented out; its
// formula regenerates both shipped code files bit-for-bit (tests/test_code_model.py).
#pragma once
#include <string>
#include <vector>

#include "Quantum_LDPC_Code.h"

class QC_LDPC_CSS {
public:
    QC_LDPC_CSS(int J, int K, int L, int P, int sigma, int tau)
    {
        qec_code* h = qec_code_generate(J, K, L, P, sigma, tau);
        if (!h) throw std::string(qec_last_error());
        code_ = std::make_shared<Quantum_LDPC_Code>(h);
    }
    const Quantum_LDPC_Code& code() const { return *code_; }
    // exponent tables HC (J x L) and HD (K x L), QEC_LDPC_CSS.cu:43-90
    std::vector<int> HC() const { return exps(0, code_->J); }
    std::vector<int> HD() const { return exps(1, code_->K); }

private:
    std::shared_ptr<Quantum_LDPC_Code> code_;
    std::vector<int> exps(int sector, int R) const
    {
        std::vector<int> e((size_t)R * code_->L);
        qec_code_exponents(code_->handle(), sector, e.data());
        return e;
    }
};
