"""Legacy Flask API (reference path deploy.py:1-54): GET / and POST /predict on port 5000.
Body: JSON dict keyed by column name -> {"prediction", "fraud_probability" (4 dp), "alert": p > 0.8}."""
import numpy as np
from flask import Flask, jsonify, request

from fraud_detection_amd.serve.engine import InferenceEngine

app = Flask(__name__)
engine = InferenceEngine.from_paths("models/logistic_model.joblib", "models/scaler.joblib",
                                    "models/feature_names.json")
columns = engine.feature_names


@app.after_request
def cors(resp):  # flask_cors is not installed; permissive CORS like the reference's CORS(app)
    resp.headers["Access-Control-Allow-Origin"] = "*"
    resp.headers["Access-Control-Allow-Headers"] = "Content-Type"
    return resp


@app.route("/", methods=["GET"])
def index():
    return jsonify({"msg": "Fraud Detection API is live"}), 200


@app.route("/predict", methods=["POST"])
def predict():
    try:
        data = request.json or request.form.to_dict()
        row = np.asarray([[float(data.get(c, "nan")) for c in columns]], dtype=np.float32)
        if not np.isfinite(row).all():
            raise ValueError("missing or non-numeric features")
        pred, prob = engine.predict(row)
        p = float(prob[0])
        return jsonify({"prediction": int(pred[0]), "fraud_probability": round(p, 4), "alert": p > 0.8}), 200
    except Exception as e:  # noqa: BLE001 - reference returns 500 {"error": ...}
        return jsonify({"error": str(e)}), 500


if __name__ == "__main__":
    app.run(debug=False, port=5000)
